# Phase F walk unroll (slab blocks per refill check) at the <24, 32> default: variants 57 / 58 /
# 59 = unroll 3 / 5 / 6 of an experiment library (build_exp/unr), interleaved with the default.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export DMF_LIB=depth-map-fusion-utils_amd/build_exp/unr/libdmf.so
SETS="-;DMF_FUSE_VARIANT=57;DMF_FUSE_VARIANT=58;DMF_FUSE_VARIANT=59;-;DMF_FUSE_VARIANT=57;DMF_FUSE_VARIANT=58;DMF_FUSE_VARIANT=59" timeout -k 10 400 bash tools/gpu_envsweep.sh || exit 1
echo SWEEPOK
