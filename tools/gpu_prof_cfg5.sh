# Config 5's per-GPU shard (1280x720, 1024^3, 256 poses) pipelined under a kernel trace:
# how much of passes A and B runs beside phase F at > 8192 bricks.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/prof_cfg5
mkdir -p $OUT
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o run -- python3 tools/exp_fuse.py --tag cfg5 --grid 1024 --image 1280x720 --poses 256 --calls 6 > $OUT/kt.json 2> $OUT/kt.err || { echo KTFAIL; tail -5 $OUT/kt.err; exit 1; }
cat $OUT/kt.json
python3 tools/kt_timeline.py $OUT/kt 2 | tail -14
echo CFG5OK
