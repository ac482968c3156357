# Phase F parameter sweep ($VARIANTS): bench lines only (no trace), alternating with the default.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/fs
for V in ${VARIANTS:-0}; do
  DMF_FUSE_VARIANT=$V timeout -k 10 200 python3 bench.py --steps 100 --warmup 3 --pmc off --cpu-frames 0 --cpu-reverse-poses 0 --no-secondary ${BENCHARGS} > gpurun_out/fs/v$V.json 2> gpurun_out/fs/v$V.err || { echo BENCHFAIL $V; tail gpurun_out/fs/v$V.err; exit 2; }
  python3 -c "import json; d=json.load(open('gpurun_out/fs/v$V.json')); print('$V', '%.3f'%d['roofline']['kernel_ms'], d['roofline']['kernel'])"
done
echo ALLOK
