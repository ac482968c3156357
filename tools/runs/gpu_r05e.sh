#!/bin/bash
# Round 5: full GPU suite, the headline bench line and config 2 (fused small-grid layout
# kernel, ctl memset dropped), plus the pipelined config-2 kernel trace.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r05e
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo TESTFAIL; tail -40 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
timeout -k 10 300 python bench.py --grid 256 --poses-per-gpu 64 --pmc auto > $O/config2.json 2> $O/config2.err || { echo CFG2FAIL; tail -20 $O/config2.err; exit 2; }
python tools/show_bench.py $O/config2.json | head -3
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || { echo BENCHFAIL; tail -30 $O/bench.err; exit 3; }
python tools/show_bench.py $O/bench.json
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_cfg2 -o run -- python3 tools/exp_fuse.py --grid 256 --poses 64 --calls 30 --modes pipelined > /dev/null 2> $O/kt_cfg2.err || { echo KTFAIL; exit 4; }
echo ALLOK
