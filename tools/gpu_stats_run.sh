# Bench lines of the DMF_EXP_STATS experiment library (phase timers) for fusion variants $VARIANTS
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/stats
for V in ${VARIANTS:-0}; do
  DMF_LIB=depth-map-fusion-utils_amd/build_exp/${EXP:-stats}/libdmf.so DMF_FUSE_VARIANT=$V timeout -k 10 200 python3 bench.py --steps 3 --warmup 1 --cpu-frames 0 --no-secondary ${BENCHARGS} > gpurun_out/stats/v$V.json 2> gpurun_out/stats/v$V.err || { echo BENCHFAIL $V; tail gpurun_out/stats/v$V.err; exit 2; }
  python3 -c "import json; d=json.load(open('gpurun_out/stats/v$V.json')); print('$V', d['roofline']['kernel_ms'], json.dumps(d['fuse_diagnostics']))"
done
echo ALLOK
