#!/bin/bash
# Round 6: reverse-march burst re-swept after the next-sample precompute at 6 waves (items /
# refill / burst: product 64/8/64, b48 64/8/48, b96 64/8/96, b128 64/8/128); alternating on the
# bench's secondary workload (512^3, 128 poses), kernels 0 (default) and 5.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r06ah
mkdir -p $O
B=depth-map-fusion-utils_amd
for rep in 1 2 3; do
  for lib in product b48 b96 b128; do
    L=$B/build/libdmf.so; [ $lib != product ] && L=$B/build_exp/$lib/libdmf.so
    DMF_LIB=$L timeout -k 10 300 python3 tools/exp_reverse.py 0,5,0 > $O/rev_${lib}_$rep.json 2> $O/rev_${lib}_$rep.err || { echo "FAIL $lib"; tail -5 $O/rev_${lib}_$rep.err; exit 3; }
    python3 -c "import json; d=json.load(open('$O/rev_${lib}_$rep.json')); print('$lib', {k: round(v,3) for k,v in d.items() if k.startswith('ms_')}, {k: v for k,v in d.items() if k.startswith('samples_')}, d['masks_equal'], d['good_digest_match'], d['good_digest_expected'])"
  done
done
echo ALLOK
