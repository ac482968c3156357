# brick-owned fusion: parity tests, then a bench line per variant (A/B), then a kernel trace
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "brick or fuse_parity" -x -v --timeout 120 --timeout-method thread > gpurun_out/bk_test.log 2>&1 || { echo TESTFAIL; exit 1; }
for V in ${VARIANTS:-40 41 42 43}; do
  DMF_FUSE_VARIANT=$V timeout -k 10 200 python bench.py --steps 3 --warmup 1 --cpu-frames 0 --no-secondary > gpurun_out/bk_bench_$V.json 2> gpurun_out/bk_bench_$V.err || { echo BENCHFAIL $V; exit 2; }
done
if [ -n "$PROF" ]; then
  export TMPDIR=/tmp DMF_FUSE_VARIANT=$PROF
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/bk_prof -o run -- python3 bench.py --steps 3 --warmup 1 --cpu-frames 0 --no-secondary > gpurun_out/bk_prof.json 2> gpurun_out/bk_prof.err || { echo PROFFAIL; exit 3; }
fi
echo ALLOK
