#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r05i
mkdir -p $O
DMF_LIB=depth-map-fusion-utils_amd/build_exp/layoutdbg/libdmf.so timeout -k 10 120 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 100 --timeout-method thread -k "multi_batch" > $O/dbg.log 2>&1
echo "rc $?"
grep -m 40 "B over\|B count" $O/dbg.log
tail -3 $O/dbg.log
