#!/bin/bash
# Round 5: pass B at 96 VGPRs (the long-ray replay without 64-bit walk state: 5 waves per
# SIMD instead of 4) vs the previous build (b116); then the fusion parity tests that cover
# long rays, and the bench's two-rank launcher rehearsal under gloo (the RCCL-agreement step).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r05p
N_LIBS="b116" O_DIR=$O bash tools/runs/gpu_r05n.sh || exit $?
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_pipeline.py tests/test_gpu_parity.py -k "fuse or long or pipelined or timed" > $O/tests.log 2>&1 || { echo FAIL tests; tail -20 $O/tests.log; exit 4; }
tail -2 $O/tests.log
DMF_BENCH_BACKEND=gloo timeout -k 10 400 python3 bench.py --gpus 2 --steps 20 --warmup 3 --pmc off --no-secondary --cpu-frames 0 --serial-ref off > $O/bench_n2_gloo.json 2> $O/bench_n2_gloo.err || { echo DISTFAIL; tail -30 $O/bench_n2_gloo.err; exit 5; }
python3 -c "import json; d=json.load(open('$O/bench_n2_gloo.json')); print(d['n_gpus'], d['config']['global_poses'], d['digest_match'], d['rccl'])"
echo ALLOK
