# Pipelined fusion: parity tests, then the headline bench pipelined vs serial,
# and the phase-F flush rewrite against the previous build (DMF_LIB=build_exp/libdmf_oldflush.so).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_pipeline.py -x -v --timeout 180 --timeout-method thread > gpurun_out/pipe_tests.log 2>&1 || { echo TESTFAIL; tail -40 gpurun_out/pipe_tests.log; exit 1; }
tail -4 gpurun_out/pipe_tests.log
OLD=depth-map-fusion-utils_amd/build_exp/libdmf_oldflush.so
NEW=depth-map-fusion-utils_amd/build/libdmf.so
for mode in new:0:1 old:0:1 new:1:1 new:1:2 new:0:1 old:0:1 new:1:1 new:1:2; do
  IFS=: read lib pipe lv <<< "$mode"
  L=$NEW; [ $lib = old ] && L=$OLD
  DMF_LIB=$L DMF_BENCH_PIPE=$pipe DMF_BK_STAGE=$lv timeout -k 10 200 python bench.py --steps ${STEPS:-400} --no-secondary --pmc off --cpu-frames 0 ${BENCH_ARGS:-} > gpurun_out/b_$lib$pipe$lv.json 2> gpurun_out/b_$lib$pipe$lv.err || { echo BENCHFAIL; tail -20 gpurun_out/b_$lib$pipe$lv.err; exit 3; }
  python -c "import json;d=json.load(open('gpurun_out/b_$lib$pipe$lv.json'));r=d['roofline'];print('$lib pipe=$pipe stage=$lv', round(d['value']/1e12,4), round(d['ms_per_step'],4), round(r['kernel_ms'],4), round(r['frac'],4), r.get('serial_call_ms'), round(d['step_breakdown_ms']['fuse'],4), d['logodds_digest'])"
done
echo ALLOK
