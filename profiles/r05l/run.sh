#!/bin/bash
# Round 5: pass A's issue priority beside phase F (s_setprio 1/2/3) with pass B held until the
# previous call's phase F ends, vs the product; 512^3 x 128 and 256^3 x 64 pipelined calls.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r05l
mkdir -p $O
B=depth-map-fusion-utils_amd
for rep in 1 2; do
  for lib in product bafterf aprio1 aprio2 aprio3; do
    L=$B/build/libdmf.so; [ $lib != product ] && L=$B/build_exp/$lib/libdmf.so
    DMF_LIB=$L timeout -k 10 200 python3 tools/exp_fuse.py --tag $lib --calls 60 --modes pipelined > $O/c4_${lib}_$rep.json 2> $O/c4_${lib}_$rep.err || { echo "FAIL $lib"; tail -5 $O/c4_${lib}_$rep.err; exit 3; }
    DMF_LIB=$L timeout -k 10 200 python3 tools/exp_fuse.py --tag $lib --grid 256 --poses 64 --calls 150 --modes pipelined > $O/c2_${lib}_$rep.json 2> $O/c2_${lib}_$rep.err || { echo "FAIL $lib"; tail -5 $O/c2_${lib}_$rep.err; exit 3; }
    python3 -c "import json; b=json.load(open('$O/c4_${lib}_$rep.json')); c=json.load(open('$O/c2_${lib}_$rep.json')); print('$lib', round(b['pipelined_ms'],4), b['digest']=='36708f70245952ff', round(c['pipelined_ms'],4), c['digest']=='605646542483b87f')"
  done
done
DMF_LIB=$B/build_exp/aprio2/libdmf.so timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_aprio2 -o run -- python3 tools/exp_fuse.py --calls 30 --modes pipelined > /dev/null 2> $O/kt.err || { echo KTFAIL; exit 4; }
echo ALLOK
