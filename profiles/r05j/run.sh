#!/bin/bash
# Round 5: reverseRayTraceFast queue shape re-swept on the per-XCD workgroup-unit kernel
# (refill threshold / burst length at 64 items per wave), alternating with the product.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r05j
mkdir -p $O
B=depth-map-fusion-utils_amd
for rep in 1 2; do
  for lib in product rev_r4_b16 rev_r8_b8 rev_r8_b24 rev_r16_b16 rev_r8_b32 rev_r12_b16; do
    L=$B/build/libdmf.so; [ $lib != product ] && L=$B/build_exp/$lib/libdmf.so
    DMF_LIB=$L timeout -k 10 120 python3 tools/exp_reverse.py 0 > $O/${lib}_$rep.json 2> $O/${lib}_$rep.err || { echo "FAIL $lib"; tail -5 $O/${lib}_$rep.err; exit 3; }
    python3 -c "import json; b=json.load(open('$O/${lib}_$rep.json')); print('$lib', round(b['ms_kernel0'],4), b['samples_kernel0'])"
  done
done
echo ALLOK
