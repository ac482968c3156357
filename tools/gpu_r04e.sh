# Round-4 run e: pipelined stage order A/B, reverse queue burst sweep.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/gpu_exp_stage.sh || exit 1
REV_LIBS="r512_8_16 r512_8_32 r512_4_16 r256_8_16" bash tools/gpu_exp_rev.sh || exit 2
echo R04EOK
