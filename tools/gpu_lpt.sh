# Part order A/B (DMF_BK_LPT): brick parity tests, then bench lines with and without the
# largest-first part order at 512^3, 256^3 (config 2) and 1024^3 (config 5 shard).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/lpt
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -x -q --timeout 180 --timeout-method thread -k "brick or multi_batch or anisotropic or config2" > gpurun_out/lpt/tests.log 2>&1 || { echo TESTFAIL; tail -30 gpurun_out/lpt/tests.log; exit 1; }
tail -1 gpurun_out/lpt/tests.log
for c in "d512 --steps 100" "c2 --steps 300 --grid 256 --poses-per-gpu 64" "c5 --steps 40 --grid 1024 --poses-per-gpu 32 --image 1280x720"; do
  set -- $c; name=$1; shift
  for L in 1 0; do
    DMF_BK_LPT=$L timeout -k 10 300 python3 bench.py --warmup 3 --pmc off --cpu-frames 0 --cpu-reverse-poses 0 --no-secondary "$@" > gpurun_out/lpt/$name.$L.json 2> gpurun_out/lpt/$name.$L.err || { echo BENCHFAIL $name $L; tail gpurun_out/lpt/$name.$L.err; exit 2; }
    python3 -c "import json; d=json.load(open('gpurun_out/lpt/$name.$L.json')); print('$name lpt=$L', '%.3e'%d['value'], 'step %.3f'%d['ms_per_step'], 'fuse %.3f'%d['roofline']['kernel_ms'], 'frac %.3f'%d['roofline']['frac'])"
  done
done
echo ALLOK
