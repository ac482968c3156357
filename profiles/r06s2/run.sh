#!/bin/bash
# Round 6: pass A/B workgroups of 128 lanes below 8192 bricks (t128: pass A beside phase F with 1
# 2-wave workgroups: half of pass A's waves beside F), default span (64 packets) and span 32, vs the product
# (256 lanes, 64 packets); alternating, headline and config 2.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r06s2
mkdir -p $O
B=depth-map-fusion-utils_amd
for rep in 1 2; do
  for v in "product:" "t128:" "t128:span=32"; do
    lib=${v%%:*}; kn=${v#*:}; args=""; tag=$lib; [ -n "$kn" ] && { args="--knob $kn"; tag=${lib}_${kn/=/}; }
    L=$B/build/libdmf.so; [ $lib != product ] && L=$B/build_exp/$lib/libdmf.so
    DMF_LIB=$L timeout -k 10 200 python3 tools/exp_fuse.py --tag $tag --calls 60 $args > $O/c4_${tag}_$rep.json 2> $O/c4_${tag}_$rep.err || { echo "FAIL $tag"; tail -5 $O/c4_${tag}_$rep.err; exit 3; }
    DMF_LIB=$L timeout -k 10 200 python3 tools/exp_fuse.py --tag $tag --grid 256 --poses 64 --calls 150 $args > $O/c2_${tag}_$rep.json 2> /dev/null || { echo "FAIL $tag"; exit 3; }
    python3 -c "import json; b=json.load(open('$O/c4_${tag}_$rep.json')); c=json.load(open('$O/c2_${tag}_$rep.json')); print('$tag', round(b['serial_ms'],4), round(b['pipelined_ms'],4), b['digest']=='36708f70245952ff', round(c['serial_ms'],4), round(c['pipelined_ms'],4), c['digest']=='605646542483b87f')"
  done
done
echo ALLOK
