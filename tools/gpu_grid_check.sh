# default fusion path at 256^3 / 512^3 / 1024^3 (640x480 frames) vs forced variants
set -o pipefail
mkdir -p gpurun_out/grid
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "fuse" -x -q --timeout 120 --timeout-method thread > gpurun_out/grid/tests.log 2>&1 || { echo TESTFAIL; tail -20 gpurun_out/grid/tests.log; exit 1; }
for cfg in "1024 32 0" "1024 32 31" "256 64 0" "256 64 40" "512 128 0"; do
  set -- $cfg
  DMF_FUSE_VARIANT=$3 timeout -k 10 300 python bench.py --grid $1 --poses-per-gpu $2 --steps 2 --warmup 1 --cpu-frames 0 --no-secondary > gpurun_out/grid/g$1_v$3.json 2> gpurun_out/grid/g$1_v$3.err || { echo FAIL $cfg; tail gpurun_out/grid/g$1_v$3.err; exit 2; }
done
echo ALLOK
