#!/bin/bash
# Round 6: phase F after the slab code -- refill / unroll re-sweep and the compiler's atomic
# optimizer off (nao), against sc0 (the slab-code commit) and the product (+ refill micro-cuts).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r06b
mkdir -p $O
B=depth-map-fusion-utils_amd
LIBS="product sc0 nao rf20 rf24 u10 u12"
for rep in 1 2; do
  for lib in $LIBS; do
    L=$B/build/libdmf.so; [ $lib != product ] && L=$B/build_exp/$lib/libdmf.so
    DMF_LIB=$L timeout -k 10 200 python3 tools/exp_fuse.py --tag $lib --calls 60 > $O/c4_${lib}_$rep.json 2> $O/c4_${lib}_$rep.err || { echo "FAIL $lib"; tail -5 $O/c4_${lib}_$rep.err; exit 3; }
    DMF_LIB=$L timeout -k 10 200 python3 tools/exp_fuse.py --tag $lib --grid 256 --poses 64 --calls 150 > $O/c2_${lib}_$rep.json 2> /dev/null || { echo "FAIL $lib"; exit 3; }
    python3 -c "import json; b=json.load(open('$O/c4_${lib}_$rep.json')); c=json.load(open('$O/c2_${lib}_$rep.json')); print('$lib', round(b['serial_ms'],4), round(b['pipelined_ms'],4), b['digest']=='36708f70245952ff', round(c['serial_ms'],4), round(c['pipelined_ms'],4), c['digest']=='605646542483b87f')"
  done
done
echo ALLOK
