# Round-4 run b: the GPU suite, smoke, the default bench line (+ config 2), then the pass-B
# diagnostics (tools/gpu_exp_b.sh) and the reverseRayTraceFast work-order A/B.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/gpu_r04a.sh || exit $?
OUT=gpurun_out/exp_b
mkdir -p $OUT
timeout -k 10 300 python3 tools/exp_reverse.py > $OUT/reverse.json 2> $OUT/reverse.err || { echo REVFAIL; tail -5 $OUT/reverse.err; exit 5; }
cat $OUT/reverse.json
EXP_LIBS="b_f64 b_nocount b_nostore b_noatomic" bash tools/gpu_exp_b.sh || exit 6
echo R04BOK
