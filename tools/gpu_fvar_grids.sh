# Phase F parameter variants (52 = <24, 16>, 54 = <24, 64>, 55 = refill 20, 56 = refill 28; default
# <24, 32>) at config 2 (256^3) and config 5's 1024^3 shard, interleaved with the default.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
V="-;DMF_FUSE_VARIANT=52;DMF_FUSE_VARIANT=54;DMF_FUSE_VARIANT=55;DMF_FUSE_VARIANT=56"
BENCHARGS="--grid 256 --poses-per-gpu 64" SETS="$V;$V" timeout -k 10 400 bash tools/gpu_envsweep.sh || exit 1
BENCHARGS="--grid 1024 --poses-per-gpu 32 --image 1280x720" SETS="$V;-" timeout -k 10 500 bash tools/gpu_envsweep.sh || exit 2
echo SWEEPOK
