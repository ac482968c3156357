#!/bin/bash
# Round 6: the reverse march computing the next sample while its loads are in flight (precomp:
# DMF_EXP_REV_PRECOMP=1, 7 waves with 2 VGPRs spilled; precomp6: the same held to 6 waves, no
# spill) vs the product; alternating, bench's secondary workload, kernels 0 / 5; parity tests.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r06ag
mkdir -p $O
B=depth-map-fusion-utils_amd
for rep in 1 2 3; do
  for lib in product precomp precomp6; do
    L=$B/build/libdmf.so; [ $lib != product ] && L=$B/build_exp/$lib/libdmf.so
    DMF_LIB=$L timeout -k 10 300 python3 tools/exp_reverse.py 0,5,0 > $O/rev_${lib}_$rep.json 2> $O/rev_${lib}_$rep.err || { echo "FAIL $lib"; tail -5 $O/rev_${lib}_$rep.err; exit 3; }
    python3 -c "import json; e=json.load(open('$O/rev_${lib}_$rep.json')); print('$lib', {k: round(v,3) for k,v in e.items() if k.startswith('ms_')}, e['masks_equal'], e['good_digest_match']['0'] == e['good_digest_expected'])"
  done
done
DMF_LIB=$B/build_exp/precomp6/libdmf.so timeout -k 10 600 python3 -u -m pytest tests/test_gpu_marches.py tests/test_gpu_parity.py -k "reverse or march or golden" -x -q --timeout 200 --timeout-method thread > $O/tests_precomp6.log 2>&1 || { echo FAIL tests; tail -30 $O/tests_precomp6.log; exit 4; }
tail -1 $O/tests_precomp6.log
echo ALLOK
