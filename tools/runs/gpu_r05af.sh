#!/bin/bash
# Round 5: pass A's one-step histogram aggregation, also for the hashed histogram (1024^3),
# vs the loop over every distinct brick (aloop): config 5's shard pipelined (1280x720, 1024^3,
# 256 poses) and the hashed-histogram tests.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r05af
mkdir -p $O
B=depth-map-fusion-utils_amd
for rep in 1 2; do
  for lib in product aloop; do
    L=$B/build/libdmf.so; [ $lib != product ] && L=$B/build_exp/$lib/libdmf.so
    DMF_LIB=$L timeout -k 10 400 python3 tools/exp_fuse.py --tag $lib --grid 1024 --image 1280x720 --poses 256 --calls 8 --modes pipelined > $O/c5_${lib}_$rep.json 2> $O/c5_${lib}_$rep.err || { echo "FAIL $lib"; tail -3 $O/c5_${lib}_$rep.err; exit 3; }
    python3 -c "import json; c=json.load(open('$O/c5_${lib}_$rep.json')); print('$lib', round(c['pipelined_ms'],3), c['digest'])"
  done
done
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_pipeline.py tests/test_gpu_parity.py tests/test_gpu_configs.py -k "hash or fuse or config5 or pipelined" > $O/tests.log 2>&1 || { echo FAIL tests; tail -20 $O/tests.log; exit 4; }
tail -2 $O/tests.log
echo ALLOK
