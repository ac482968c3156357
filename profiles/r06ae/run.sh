#!/bin/bash
# Round 6: the collision cost map with 2 / 4 groups of 64 depths per ballot, their occupancy loads
# in flight together (cu2 / cu4: DMF_EXP_COST_UNROLL) vs the product's one group; alternating,
# bench's secondary workload (1024 centres), maps against the oracle's digest; then the cost-map
# parity tests with cu2.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r06ae
mkdir -p $O
B=depth-map-fusion-utils_amd
for rep in 1 2; do
  for lib in product cu2 cu4; do
    L=$B/build/libdmf.so; [ $lib != product ] && L=$B/build_exp/$lib/libdmf.so
    DMF_LIB=$L timeout -k 10 300 python3 tools/exp_costmap.py 0,0 > $O/cm_${lib}_$rep.json 2> $O/cm_${lib}_$rep.err || { echo "FAIL $lib"; tail -5 $O/cm_${lib}_$rep.err; exit 3; }
    python3 -c "import json; d=json.load(open('$O/cm_${lib}_$rep.json')); print('$lib', d['ms_skip0'], d['maps_equal'], d['digest']['0'] == d.get('digest_expected'))"
  done
done
for lib in cu2 cu4; do
  DMF_LIB=$B/build_exp/$lib/libdmf.so timeout -k 10 600 python3 -u -m pytest tests/test_gpu_marches.py tests/test_gpu_parity.py -k "cost_map or will_collide or march" -x -q --timeout 200 --timeout-method thread > $O/tests_$lib.log 2>&1 || { echo FAIL tests $lib; tail -30 $O/tests_$lib.log; exit 4; }
  tail -1 $O/tests_$lib.log
done
echo ALLOK
