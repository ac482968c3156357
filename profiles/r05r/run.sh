#!/bin/bash
# Round 5 re-verification after the pass-B replay and k_reverse_x register changes: the whole
# GPU suite, smoke, then the default bench line with its PMC child kept.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r05r
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo FAIL tests; tail -30 $O/gpu_tests.log; exit 4; }
tail -2 $O/gpu_tests.log
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { echo FAIL smoke; tail -20 $O/smoke.log; exit 5; }
tail -1 $O/smoke.log
timeout -k 10 400 python3 bench.py --pmc-dir $O/pmc_child > $O/bench_default.json 2> $O/bench_default.err || { echo BENCHFAIL; tail -20 $O/bench_default.err; exit 1; }
python3 tools/show_bench.py $O/bench_default.json | head -12
echo ALLOK
