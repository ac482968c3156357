#!/bin/bash
# Round 6: (1) the forward march ended once a sample outside the volume lies past the line's exit
# from the volume grown by the margin (fexit: DMF_FWD_EXIT_END=1) vs the product, fwd kernels 0 /
# 1 / 2 and the march parity tests with fexit; (2) the reverse queue's burst re-swept past 64
# (b64 / b96 / b128 at 64 items, refill 8) vs the product's 32.  Alternating, bench's secondary
# workload.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r06ac
mkdir -p $O
B=depth-map-fusion-utils_amd
for rep in 1 2; do
  for lib in product fexit; do
    L=$B/build/libdmf.so; [ $lib != product ] && L=$B/build_exp/$lib/libdmf.so
    DMF_LIB=$L timeout -k 10 300 python3 tools/exp_forward.py 0,1,2,0 > $O/fwd_${lib}_$rep.json 2> $O/fwd_${lib}_$rep.err || { echo "FAIL $lib"; tail -5 $O/fwd_${lib}_$rep.err; exit 3; }
    python3 -c "import json; d=json.load(open('$O/fwd_${lib}_$rep.json')); print('$lib', {k: v for k,v in d.items() if k.startswith('ms_') or k.startswith('samples_')}, d['outputs_equal'], d.get('digest_match'))"
  done
  for lib in product b64 b96 b128; do
    L=$B/build/libdmf.so; [ $lib != product ] && L=$B/build_exp/$lib/libdmf.so
    DMF_LIB=$L timeout -k 10 300 python3 tools/exp_reverse.py 0,5,0 > $O/rev_${lib}_$rep.json 2> $O/rev_${lib}_$rep.err || { echo "FAIL $lib"; tail -5 $O/rev_${lib}_$rep.err; exit 3; }
    python3 -c "import json; d=json.load(open('$O/rev_${lib}_$rep.json')); print('$lib', {k: round(v,3) for k,v in d.items() if k.startswith('ms_')}, d['masks_equal'], d['good_digest_match']['0'] == d['good_digest_expected'])"
  done
done
DMF_LIB=$B/build_exp/fexit/libdmf.so timeout -k 10 600 python3 -u -m pytest tests/test_gpu_marches.py tests/test_gpu_parity.py -k "forward or march or ray_trace or golden or truncated" -x -q --timeout 200 --timeout-method thread > $O/tests_fexit.log 2>&1 || { echo FAIL tests; tail -30 $O/tests_fexit.log; exit 4; }
tail -2 $O/tests_fexit.log
echo ALLOK
