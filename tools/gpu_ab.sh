# Parity of the working build on the fusion tests, then an alternating A/B of fusion bench
# lines: build/ (new) against build_exp/$OLD (default "old"), $ROUNDS rounds.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ab
if [ -z "$NOTEST" ]; then
  timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -x -q --timeout 300 --timeout-method thread \
    -k "${TESTK:-brick or edge or multi_batch or config}" > gpurun_out/ab/tests.log 2>&1 || { echo TESTFAIL; tail -30 gpurun_out/ab/tests.log; exit 1; }
  tail -2 gpurun_out/ab/tests.log
fi
for i in $(seq 1 ${ROUNDS:-3}); do
  for E in ${OLD:-old} new; do
    if [ "$E" = new ]; then LIB=depth-map-fusion-utils_amd/build/libdmf.so; else LIB=depth-map-fusion-utils_amd/build_exp/$E/libdmf.so; fi
    DMF_LIB=$LIB timeout -k 10 200 python3 bench.py --steps ${STEPS:-300} --warmup 3 --pmc off --cpu-frames 0 --cpu-reverse-poses 0 --no-secondary ${BENCHARGS} > gpurun_out/ab/$E$i.json 2> gpurun_out/ab/$E$i.err || { echo BENCHFAIL $E; tail gpurun_out/ab/$E$i.err; exit 2; }
    python3 -c "import json; d=json.load(open('gpurun_out/ab/$E$i.json')); print('$E', '%.3f ms'%d['roofline']['kernel_ms'], '%.4e'%d['value'], 'frac %.3f'%d['roofline']['frac'])"
  done
done
echo ALLOK
