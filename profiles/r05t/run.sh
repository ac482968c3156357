#!/bin/bash
# Round 5: the chain between pass A and pass B (batch cut fast path, 16 pose-count loads in
# flight, the scan's counts in registers) vs the previous build (chain0): pipelined timelines
# at config 2 (256^3 x 64) and the headline (512^3 x 128), then the fusion parity tests.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r05t
mkdir -p $O
B=depth-map-fusion-utils_amd
for lib in product chain0; do
  L=$B/build/libdmf.so; [ $lib != product ] && L=$B/build_exp/$lib/libdmf.so
  DMF_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/kt_c2_$lib -o run -- python3 tools/exp_fuse.py --grid 256 --poses 64 --calls 60 --modes pipelined > $O/c2_$lib.json 2> $O/c2_$lib.err || { echo FAIL c2; tail -5 $O/c2_$lib.err; exit 3; }
  DMF_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/kt_c4_$lib -o run -- python3 tools/exp_fuse.py --calls 40 --modes pipelined > $O/c4_$lib.json 2> $O/c4_$lib.err || { echo FAIL c4; tail -5 $O/c4_$lib.err; exit 3; }
  python3 tools/kt_timeline.py $O/kt_c2_$lib 5 > $O/timeline_c2_$lib.txt && python3 tools/kt_timeline.py $O/kt_c4_$lib 5 > $O/timeline_c4_$lib.txt
done
for rep in 1 2; do
  for lib in product chain0; do
    L=$B/build/libdmf.so; [ $lib != product ] && L=$B/build_exp/$lib/libdmf.so
    DMF_LIB=$L timeout -k 10 200 python3 tools/exp_fuse.py --tag $lib --calls 60 --modes pipelined > $O/p_c4_${lib}_$rep.json 2> /dev/null || { echo "FAIL $lib"; exit 3; }
    DMF_LIB=$L timeout -k 10 200 python3 tools/exp_fuse.py --tag $lib --grid 256 --poses 64 --calls 150 --modes pipelined > $O/p_c2_${lib}_$rep.json 2> /dev/null || { echo "FAIL $lib"; exit 3; }
    python3 -c "import json; b=json.load(open('$O/p_c4_${lib}_$rep.json')); c=json.load(open('$O/p_c2_${lib}_$rep.json')); print('$lib', round(b['pipelined_ms'],4), b['digest']=='36708f70245952ff', round(c['pipelined_ms'],4), c['digest']=='605646542483b87f')"
  done
done
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_pipeline.py tests/test_gpu_configs.py tests/test_gpu_parity.py -k "fuse or long or pipelined or timed or config or batch" > $O/tests.log 2>&1 || { echo FAIL tests; tail -20 $O/tests.log; exit 4; }
tail -2 $O/tests.log
echo ALLOK
