#!/bin/bash
# Round 6: reverseRayTraceFast refills reading each item's hash from a Morton-ordered copy (hsort:
# DMF_REV_HSORT=1; one load independent of the slot's) vs through its slot (product: two dependent
# loads); alternating, bench's secondary workload, kernels 0 / 5; then the reverse parity tests.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r06af
mkdir -p $O
B=depth-map-fusion-utils_amd
for rep in 1 2 3; do
  for lib in product hsort; do
    L=$B/build/libdmf.so; [ $lib != product ] && L=$B/build_exp/$lib/libdmf.so
    DMF_LIB=$L timeout -k 10 300 python3 tools/exp_reverse.py 0,5,0 > $O/rev_${lib}_$rep.json 2> $O/rev_${lib}_$rep.err || { echo "FAIL $lib"; tail -5 $O/rev_${lib}_$rep.err; exit 3; }
    python3 -c "import json; e=json.load(open('$O/rev_${lib}_$rep.json')); print('$lib', {k: round(v,3) for k,v in e.items() if k.startswith('ms_')}, e['masks_equal'], e['good_digest_match']['0'] == e['good_digest_expected'])"
  done
done
DMF_LIB=$B/build_exp/hsort/libdmf.so timeout -k 10 600 python3 -u -m pytest tests/test_gpu_marches.py tests/test_gpu_parity.py -k "reverse or march or golden" -x -q --timeout 200 --timeout-method thread > $O/tests_hsort.log 2>&1 || { echo FAIL tests; tail -30 $O/tests_hsort.log; exit 4; }
tail -1 $O/tests_hsort.log
echo ALLOK
