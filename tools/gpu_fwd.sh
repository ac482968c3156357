# Forward-march parity tests, then the bench's secondary forward line with and without skipping
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/fwd
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_compat.py tests/test_reference_driver.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/fwd/tests.log 2>&1 || { echo TESTFAIL; tail -30 gpurun_out/fwd/tests.log; exit 1; }
tail -2 gpurun_out/fwd/tests.log
for S in 1 0; do
  DMF_FWD_SKIP=$S timeout -k 10 300 python bench.py --steps 2 --warmup 1 --cpu-frames 0 --cpu-reverse-poses 0 --pmc off > gpurun_out/fwd/b$S.json 2> gpurun_out/fwd/b$S.err || { echo BENCHFAIL; tail gpurun_out/fwd/b$S.err; exit 2; }
  python3 -c "import json; d=json.load(open('gpurun_out/fwd/b$S.json'))['secondary']['forward_first_hits']; print('skip=$S', '%.3f ms'%d['ms_per_batch'], '%.3e samples/s'%d['march_samples_per_s'], '%.0f Mrays/s'%d['mrays_per_s'])"
done
echo ALLOK
