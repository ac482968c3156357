# Round-4 run o: the full GPU suite + smoke + bench + config 2 (tools/runs/gpu_r04a.sh), then a
# reverseRayTraceFast queue-shape sweep around the default 128 / 8 / 16.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
TAG=r04o bash tools/runs/gpu_r04a.sh || exit 1
REV_LIBS="r64_8_16 r192_8_16 r128_4_16 r128_16_16 r128_8_24" bash tools/gpu_exp_rev.sh || exit 2
echo R04OOK
