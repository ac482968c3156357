#!/bin/bash
# Round 5: fused small-grid layout kernel (pose pairs staged in LDS): 256^3 parity subset,
# config 2 kernel trace and bench lines.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r05f
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_pipeline.py tests/test_gpu_configs.py tests/test_gpu_parity.py -m gpu -x -v --timeout 240 --timeout-method thread -k "256 or config2 or multi_batch or oracle_128 or edge_cases" > $O/tests.log 2>&1 || { echo TESTFAIL; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_cfg2 -o run -- python3 tools/exp_fuse.py --grid 256 --poses 64 --calls 30 --modes pipelined > /dev/null 2> $O/kt_cfg2.err || { echo KTFAIL; exit 4; }
for r in 1 2; do
timeout -k 10 300 python bench.py --grid 256 --poses-per-gpu 64 --pmc off --cpu-frames 0 --no-secondary > $O/config2_$r.json 2> $O/config2_$r.err || { echo CFG2FAIL; tail -20 $O/config2_$r.err; exit 2; }
python tools/show_bench.py $O/config2_$r.json | head -2
done
echo ALLOK
