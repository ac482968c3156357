# finalize rewrite: fusion/finalize parity tests, then bench steps at 512^3 and 1024^3
set -o pipefail
mkdir -p gpurun_out/fin
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "fuse or golden" -x -q --timeout 120 --timeout-method thread > gpurun_out/fin/tests.log 2>&1 || { echo TESTFAIL; tail -20 gpurun_out/fin/tests.log; exit 1; }
timeout -k 10 300 python bench.py --grid 1024 --poses-per-gpu 32 --steps 2 --warmup 1 --cpu-frames 0 --no-secondary > gpurun_out/fin/g1024.json 2> gpurun_out/fin/g1024.err || { echo FAIL1024; exit 2; }
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --cpu-frames 0 --no-secondary > gpurun_out/fin/g512.json 2> gpurun_out/fin/g512.err || { echo FAIL512; exit 3; }
echo ALLOK
