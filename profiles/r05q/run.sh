#!/bin/bash
# Round 5: the march kernels at a higher occupancy (experiment builds: k_reverse_x held to 72 /
# 64 VGPRs = 7 / 8 waves per SIMD (rw7 / rw8), k_forward to 72 (fw7); the product: 76 / 79 =
# 6 waves), on bench.py's secondary workload; masks / outputs compared within each run.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r05q
mkdir -p $O
B=depth-map-fusion-utils_amd
for rep in 1 2; do
  for lib in product rw7 rw8; do
    L=$B/build/libdmf.so; [ $lib != product ] && L=$B/build_exp/$lib/libdmf.so
    DMF_LIB=$L timeout -k 10 300 python3 tools/exp_reverse.py 0,0 > $O/rev_${lib}_$rep.json 2> $O/rev_${lib}_$rep.err || { echo "FAIL rev $lib"; tail -5 $O/rev_${lib}_$rep.err; exit 3; }
    python3 -c "import json; d=json.load(open('$O/rev_${lib}_$rep.json')); print('rev $lib', round(d['ms_kernel0'],4), d['masks_equal'], d.get('good_digest_match'), d.get('good_digest_expected'))"
  done
  for lib in product fw7; do
    L=$B/build/libdmf.so; [ $lib != product ] && L=$B/build_exp/$lib/libdmf.so
    DMF_LIB=$L timeout -k 10 300 python3 tools/exp_forward.py 0,0 > $O/fwd_${lib}_$rep.json 2> $O/fwd_${lib}_$rep.err || { echo "FAIL fwd $lib"; tail -5 $O/fwd_${lib}_$rep.err; exit 3; }
    cat $O/fwd_${lib}_$rep.json
  done
done
echo ALLOK
