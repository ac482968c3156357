#!/bin/bash
# Round 6: both marches with the brick's distance byte loaded together with the occupancy word
# (early: DMF_EXP_EARLY_BDIST=1; the product loads it after the occupancy test) -- one memory
# latency per empty sample instead of two; alternating, bench's secondary workload; then the
# march parity tests with the experiment library.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r06ad
mkdir -p $O
B=depth-map-fusion-utils_amd
for rep in 1 2; do
  for lib in product early; do
    L=$B/build/libdmf.so; [ $lib != product ] && L=$B/build_exp/$lib/libdmf.so
    DMF_LIB=$L timeout -k 10 300 python3 tools/exp_forward.py 0,0 > $O/fwd_${lib}_$rep.json 2> $O/fwd_${lib}_$rep.err || { echo "FAIL $lib"; tail -5 $O/fwd_${lib}_$rep.err; exit 3; }
    DMF_LIB=$L timeout -k 10 300 python3 tools/exp_reverse.py 0,5,0 > $O/rev_${lib}_$rep.json 2> $O/rev_${lib}_$rep.err || { echo "FAIL $lib"; tail -5 $O/rev_${lib}_$rep.err; exit 3; }
    python3 -c "import json; d=json.load(open('$O/fwd_${lib}_$rep.json')); e=json.load(open('$O/rev_${lib}_$rep.json')); print('$lib', 'fwd', d['ms_fwd0'], d.get('digest_match'), 'rev', {k: round(v,3) for k,v in e.items() if k.startswith('ms_')}, e['good_digest_match']['0'] == e['good_digest_expected'])"
  done
done
DMF_LIB=$B/build_exp/early/libdmf.so timeout -k 10 600 python3 -u -m pytest tests/test_gpu_marches.py tests/test_gpu_parity.py -k "forward or march or reverse or ray_trace or golden or truncated" -x -q --timeout 200 --timeout-method thread > $O/tests_early.log 2>&1 || { echo FAIL tests; tail -30 $O/tests_early.log; exit 4; }
tail -2 $O/tests_early.log
echo ALLOK
