# Config 5's real per-GPU shard (1280x720, 1024^3, 256 poses = 2048 / 8 GPUs): bench line with
# live PMC, then a kernel trace of the same workload (profiles/r03_cfg5/).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/cfg5
mkdir -p "$OUT"
ARGS="--grid 1024 --poses-per-gpu 256 --image 1280x720"
timeout -k 10 500 python3 bench.py --steps 8 --warmup 2 $ARGS > "$OUT/config5shard.json" 2> "$OUT/config5shard.err" || { echo BENCHFAIL; tail "$OUT/config5shard.err"; exit 1; }
python3 tools/show_bench.py "$OUT/config5shard.json"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kt" -o run -- python3 bench.py --steps 4 --warmup 1 --cpu-frames 0 --cpu-reverse-poses 0 --pmc off --no-secondary $ARGS > "$OUT/bench_kt.json" 2> "$OUT/bench_kt.err" || { echo KTFAIL; tail "$OUT/bench_kt.err"; exit 2; }
python3 tools/kt_summary.py "$OUT" | grep -E "k_bk|k_fuse|k_fin" || exit 3
echo CFG5OK
