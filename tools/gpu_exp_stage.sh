# Pipelined stage order A/B (DMF_KNOB_STAGE_ORDER): one staging stream vs pass A on its own
# stream, kernel trace per run for tools/kt_timeline.py; digests must equal tests/golden.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/exp_stage
mkdir -p $OUT
for so in ${STAGE_ORDERS:-1 2}; do
  echo "== stage_order $so"
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt_so$so -o run -- python3 tools/exp_fuse.py --tag so$so --calls 20 --modes pipelined --knob stage_order=$so > $OUT/so$so.json 2> $OUT/so$so.err || { echo "FAIL $so"; tail -5 $OUT/so$so.err; exit 1; }
  cat $OUT/so$so.json
  python3 tools/kt_timeline.py $OUT/kt_so$so > $OUT/timeline_so$so.txt 2>&1 && tail -12 $OUT/timeline_so$so.txt
done
echo STAGEOK
