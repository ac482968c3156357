#!/bin/bash
# Round 6: reverse march, the centroid test by occupancy bit (cob; 68 VGPRs, 7 waves) and the same at
# 8 waves per SIMD (cob8: 64 VGPRs, no spill) vs the product; alternating on the bench's secondary
# workload (512^3, 128 poses), kernels 0 (default), 5, 3; then the reverse parity tests with cob8.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r06aa
mkdir -p $O
B=depth-map-fusion-utils_amd
for rep in 1 2; do
  for lib in product cob cob8; do
    L=$B/build/libdmf.so; [ $lib != product ] && L=$B/build_exp/$lib/libdmf.so
    DMF_LIB=$L timeout -k 10 300 python3 tools/exp_reverse.py 0,5,3,0 > $O/rev_${lib}_$rep.json 2> $O/rev_${lib}_$rep.err || { echo "FAIL $lib"; tail -5 $O/rev_${lib}_$rep.err; exit 3; }
    python3 -c "import json; d=json.load(open('$O/rev_${lib}_$rep.json')); print('$lib', {k: round(v,3) for k,v in d.items() if k.startswith('ms_')}, {k: v for k,v in d.items() if k.startswith('samples_')}, d['masks_equal'], d['good_digest_match'], d['good_digest_expected'])"
  done
done
DMF_LIB=$B/build_exp/cob8/libdmf.so timeout -k 10 600 python3 -u -m pytest tests/test_gpu_marches.py tests/test_gpu_parity.py -k "reverse or march" -x -q --timeout 200 --timeout-method thread > $O/tests_cob8.log 2>&1 || { echo FAIL tests; tail -30 $O/tests_cob8.log; exit 4; }
tail -2 $O/tests_cob8.log
echo ALLOK
