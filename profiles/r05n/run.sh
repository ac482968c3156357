#!/bin/bash
# Round 5: pass B's occupancy (experiment builds DMF_EXP_B_WAVES = 5 / 6: the compiler keeps
# B's registers for 5 / 6 waves per SIMD, spilling the rest; the product: 116 VGPRs, 4 waves)
# vs the product; 512^3 x 128 (serial + pipelined) and 256^3 x 64 pipelined; then B's kernel
# time per library from a kernel trace of serial calls.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=${O_DIR:-gpurun_out/r05n}
mkdir -p $O
B=depth-map-fusion-utils_amd
for rep in 1 2; do
  for lib in product ${N_LIBS:-bw5 bw6}; do
    L=$B/build/libdmf.so; [ $lib != product ] && L=$B/build_exp/$lib/libdmf.so
    DMF_LIB=$L timeout -k 10 200 python3 tools/exp_fuse.py --tag $lib --calls 60 > $O/c4_${lib}_$rep.json 2> $O/c4_${lib}_$rep.err || { echo "FAIL $lib"; tail -5 $O/c4_${lib}_$rep.err; exit 3; }
    DMF_LIB=$L timeout -k 10 200 python3 tools/exp_fuse.py --tag $lib --grid 256 --poses 64 --calls 150 --modes pipelined > $O/c2_${lib}_$rep.json 2> $O/c2_${lib}_$rep.err || { echo "FAIL $lib"; tail -5 $O/c2_${lib}_$rep.err; exit 3; }
    python3 -c "import json; b=json.load(open('$O/c4_${lib}_$rep.json')); c=json.load(open('$O/c2_${lib}_$rep.json')); print('$lib', round(b['serial_ms'],4), round(b['pipelined_ms'],4), b['digest']=='36708f70245952ff', round(c['pipelined_ms'],4), c['digest']=='605646542483b87f')"
  done
done
for lib in product ${N_LIBS:-bw5 bw6}; do
  L=$B/build/libdmf.so; [ $lib != product ] && L=$B/build_exp/$lib/libdmf.so
  DMF_LIB=$L timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_$lib -o run -- python3 tools/exp_fuse.py --calls 20 --modes serial > /dev/null 2> $O/kt_$lib.err || { echo "KTFAIL $lib"; exit 4; }
done
echo ALLOK
