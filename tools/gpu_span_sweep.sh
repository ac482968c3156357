# A/B span sweep at the grids whose brick count keeps the span at its 64-packet floor
# (256^3: 512 bricks, 384^3: 1728 bricks).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
BENCHARGS="--grid 256 --poses-per-gpu 64" SETS="-;DMF_BK_SPAN=16;DMF_BK_SPAN=24;DMF_BK_SPAN=32;DMF_BK_SPAN=48;-;DMF_BK_SPAN=32" timeout -k 10 300 bash tools/gpu_envsweep.sh || exit 1
BENCHARGS="--grid 384 --poses-per-gpu 128" SETS="-;DMF_BK_SPAN=32;DMF_BK_SPAN=48;-;DMF_BK_SPAN=32" timeout -k 10 300 bash tools/gpu_envsweep.sh || exit 2
BENCHARGS="--grid 512 --poses-per-gpu 128" SETS="-;DMF_BK_SPAN=32;-;DMF_BK_SPAN=32" timeout -k 10 300 bash tools/gpu_envsweep.sh || exit 3
echo SWEEPOK
