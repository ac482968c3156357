#!/bin/bash
# Round 6 check of the committed tree after the pass-B replay change: the GPU suite, smoke, and
# the default bench line.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r06_check3}
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo FAIL tests; tail -30 $O/gpu_tests.log; exit 4; }
tail -2 $O/gpu_tests.log
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { echo FAIL smoke; tail -20 $O/smoke.log; exit 5; }
tail -1 $O/smoke.log
timeout -k 10 400 python3 bench.py > $O/bench_default.json 2> $O/bench_default.err || { echo BENCHFAIL; tail -20 $O/bench_default.err; exit 1; }
python3 tools/show_bench.py $O/bench_default.json | head -8
python3 -c "import json; b=json.load(open('$O/bench_default.json')); c=b['roofline']['companion']; print({k: c.get(k) for k in ('f_frac','f_lds_frac','f_lds_per_launch','f_valu_per_launch')})"
echo ALLOK
