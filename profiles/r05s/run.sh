#!/bin/bash
# Round 5: the collision cost map's empty-space jumps (DMF_KNOB_COST_SKIP 0) vs the plain
# 64-depth groups (-1) on the bench's secondary workload, then the cost-map parity tests.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r05s
mkdir -p $O
timeout -k 10 300 python3 tools/exp_costmap.py 0,-1,0,-1 > $O/costmap.json 2> $O/costmap.err || { echo FAIL costmap; tail -5 $O/costmap.err; exit 3; }
cat $O/costmap.json
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_marches.py -k "collide or cost or marches" > $O/tests.log 2>&1 || { echo FAIL tests; tail -20 $O/tests.log; exit 4; }
tail -2 $O/tests.log
echo ALLOK
