#!/bin/bash
# Round 5: 16^3-cell bricks (experiment build DMF_EXP_BRICK_LOG=4, build_exp/brick16) vs the
# product's 32^3 at config 2 (256^3, 64 frames) and the headline (512^3, 128 frames):
# pipelined and serial calls, alternating, digests vs tests/golden/fusion_digests.json.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r05d
mkdir -p $O
EXP=depth-map-fusion-utils_amd/build_exp/brick16/libdmf.so
for rep in 1 2; do
  for lib in product brick16; do
    L=""; [ $lib = brick16 ] && L=$EXP
    DMF_LIB=${L:-depth-map-fusion-utils_amd/build/libdmf.so} timeout -k 10 200 python3 tools/exp_fuse.py --tag $lib --grid 256 --poses 64 --calls 100 > $O/cfg2_${lib}_$rep.json 2> $O/cfg2_${lib}_$rep.err || { echo "FAIL cfg2 $lib"; tail -5 $O/cfg2_${lib}_$rep.err; exit 3; }
    python3 -c "import json; b=json.load(open('$O/cfg2_${lib}_$rep.json')); print('cfg2', '$lib', {k: v for k, v in b.items() if 'ms' in k}, b['digest']=='605646542483b87f')"
  done
done
for lib in product brick16; do
  L=""; [ $lib = brick16 ] && L=$EXP
  DMF_LIB=${L:-depth-map-fusion-utils_amd/build/libdmf.so} timeout -k 10 200 python3 tools/exp_fuse.py --tag $lib --grid 512 --poses 128 --calls 40 > $O/c4_${lib}.json 2> $O/c4_${lib}.err || { echo "FAIL c4 $lib"; tail -5 $O/c4_${lib}.err; exit 4; }
  python3 -c "import json; b=json.load(open('$O/c4_${lib}.json')); print('c4', '$lib', {k: v for k, v in b.items() if 'ms' in k}, b['digest']=='36708f70245952ff')"
done
# kernel trace of config 2 with each library
for lib in product brick16; do
  L=""; [ $lib = brick16 ] && L=$EXP
  DMF_LIB=${L:-depth-map-fusion-utils_amd/build/libdmf.so} timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_cfg2_$lib -o run -- python3 tools/exp_fuse.py --tag $lib --grid 256 --poses 64 --calls 30 --modes pipelined > /dev/null 2> $O/kt_cfg2_$lib.err || { echo "FAIL kt $lib"; exit 5; }
done
echo ALLOK
