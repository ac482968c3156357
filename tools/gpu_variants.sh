# Fusion parity tests, then a bench line + kernel trace per fusion variant ($VARIANTS, default 40).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/var
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "${TESTK:-fuse or brick or dda}" > gpurun_out/var/tests.log 2>&1 || { echo TESTFAIL; tail -30 gpurun_out/var/tests.log; exit 1; }
for V in ${VARIANTS:-40}; do
  DMF_FUSE_VARIANT=$V timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/var/v$V -o run -- python3 bench.py --steps 5 --warmup 2 --cpu-frames 0 --no-secondary ${BENCHARGS} > gpurun_out/var/v$V.json 2> gpurun_out/var/v$V.err || { echo BENCHFAIL $V; tail gpurun_out/var/v$V.err; exit 2; }
  python3 -c "import json,sys; d=json.load(open('gpurun_out/var/v$V.json')); print('$V', '%.3e'%d['value'], '%.3f'%d['roofline']['kernel_ms'], '%.3f'%d['roofline']['frac'])"
done
for V in ${VARIANTS:-40}; do grep -h -E "k_bk|k_fuse_l" gpurun_out/var/v$V/*kernel_stats.csv | awk -F'","' -v v=$V '{printf "%s %s avg_ms=%.3f\n", v, substr($1,1,40), $4/1e6}'; done
echo ALLOK
