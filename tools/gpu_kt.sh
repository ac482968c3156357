# Kernel trace (rocprofv3 --kernel-trace --stats) of a short bench run + the bench's
# secondary kernel timings; outputs under gpurun_out/kt_$TAG.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-r03}
OUT=gpurun_out/kt_$TAG
mkdir -p "$OUT"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kt" -o run -- python3 bench.py --steps 20 --warmup 2 --cpu-frames 0 --cpu-reverse-poses 0 --pmc off ${BENCHARGS} > "$OUT/bench_kt.json" 2> "$OUT/bench_kt.err" || { echo KTFAIL; tail "$OUT/bench_kt.err"; exit 1; }
python3 tools/kt_summary.py "$OUT" || exit 2
python3 tools/show_bench.py "$OUT/bench_kt.json"
echo KT_OK
