#!/bin/bash
# Round 6: forward-march jumps without evaluating the landing sample (fwdnv:
# DMF_FWD_VERIFY_JUMPS=0; the line's point at the landing checked against the cube shrunk by
# twice the margin) vs the product (which has the reverse march's unchecked jumps); alternating,
# bench's secondary workload (128 poses x 640x480, 512^3), fwd kernels 0 / 1 / 2; then the march
# parity tests with the experiment library.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r06z
mkdir -p $O
B=depth-map-fusion-utils_amd
for rep in 1 2; do
  for lib in product fwdnv; do
    L=$B/build/libdmf.so; [ $lib != product ] && L=$B/build_exp/$lib/libdmf.so
    DMF_LIB=$L timeout -k 10 300 python3 tools/exp_forward.py 0,1,2,0 > $O/fwd_${lib}_$rep.json 2> $O/fwd_${lib}_$rep.err || { echo "FAIL $lib"; tail -5 $O/fwd_${lib}_$rep.err; exit 3; }
    python3 -c "import json; d=json.load(open('$O/fwd_${lib}_$rep.json')); print('$lib', {k: v for k,v in d.items() if k.startswith('ms_') or k.startswith('samples_')}, d['outputs_equal'], d.get('digest_match'))"
  done
done
DMF_LIB=$B/build_exp/fwdnv/libdmf.so timeout -k 10 600 python3 -u -m pytest tests/test_gpu_marches.py tests/test_gpu_parity.py -k "forward or march or reverse or ray_trace or golden or truncated" -x -q --timeout 200 --timeout-method thread > $O/tests_fwdnv.log 2>&1 || { echo FAIL tests; tail -30 $O/tests_fwdnv.log; exit 4; }
tail -2 $O/tests_fwdnv.log
echo ALLOK
