#!/bin/bash
# Round 5: reverseRayTraceFast with the march's geometry (Geom, DevVol) re-read from the
# kernarg segment at each burst (revkarg: SGPR spills 89 -> 43, v_readlane 182 -> 59, VALU
# 1094 -> 924 in the compiled k_reverse_x) vs the product; oracle digest of the good masks.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r05aj
mkdir -p $O
B=depth-map-fusion-utils_amd
for rep in 1 2 3; do
  for lib in product revkarg; do
    L=$B/build/libdmf.so; [ $lib != product ] && L=$B/build_exp/$lib/libdmf.so
    DMF_LIB=$L timeout -k 10 120 python3 tools/exp_reverse.py 0 > $O/${lib}_$rep.json 2> $O/${lib}_$rep.err || { echo "FAIL $lib"; tail -5 $O/${lib}_$rep.err; exit 3; }
    python3 -c "import json; b=json.load(open('$O/${lib}_$rep.json')); print('$lib', {k: v for k, v in b.items() if k.startswith('ms_') or k.startswith('good_digest')})"
  done
done
echo ALLOK
