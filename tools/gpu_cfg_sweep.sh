# Part-cap / A-B span sweep on the smaller-than-anchor BASELINE configs (config 2 at 256^3,
# config 5's 1024^3 shard): fusion kernel time per setting, twice, interleaved.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
BENCHARGS="--grid 256 --poses-per-gpu 64" SETS="-;DMF_BK_PART_MAX=49152;DMF_BK_PART_MAX=32768;DMF_BK_PART_MAX=16384;DMF_BK_SPAN=32;-;DMF_BK_PART_MAX=32768;DMF_BK_SPAN=32" timeout -k 10 400 bash tools/gpu_envsweep.sh || exit 1
BENCHARGS="--grid 1024 --poses-per-gpu 32 --image 1280x720" SETS="-;DMF_BK_SPAN=256;DMF_BK_SPAN=1024;DMF_BK_PART_MAX=32768;-;DMF_BK_SPAN=256" timeout -k 10 500 bash tools/gpu_envsweep.sh || exit 2
echo SWEEPOK
