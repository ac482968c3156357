#!/bin/bash
# Round 6: phase F walks S whole slabs with one ownership test per slab and adds L's slab at
# adoption (slab code, dmf_brick.hpp slab_code) vs round 5's three per-cell thresholds (r5f):
# alternating A/B at the headline and config 2, both bench lines (F VALU per launch from the
# PMC child, F ms from its kernel trace), then the fusion GPU tests on the new build.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r06a
mkdir -p $O
B=depth-map-fusion-utils_amd
for rep in 1 2; do
  for lib in product r5f; do
    L=$B/build/libdmf.so; [ $lib != product ] && L=$B/build_exp/$lib/libdmf.so
    DMF_LIB=$L timeout -k 10 200 python3 tools/exp_fuse.py --tag $lib --calls 60 > $O/c4_${lib}_$rep.json 2> $O/c4_${lib}_$rep.err || { echo "FAIL $lib"; tail -5 $O/c4_${lib}_$rep.err; exit 3; }
    DMF_LIB=$L timeout -k 10 200 python3 tools/exp_fuse.py --tag $lib --grid 256 --poses 64 --calls 150 > $O/c2_${lib}_$rep.json 2> /dev/null || { echo "FAIL $lib"; exit 3; }
    python3 -c "import json; b=json.load(open('$O/c4_${lib}_$rep.json')); c=json.load(open('$O/c2_${lib}_$rep.json')); print('$lib', round(b['serial_ms'],4), round(b['pipelined_ms'],4), b['digest']=='36708f70245952ff', round(c['serial_ms'],4), round(c['pipelined_ms'],4), c['digest']=='605646542483b87f')"
  done
done
for lib in product r5f; do
  L=$B/build/libdmf.so; [ $lib != product ] && L=$B/build_exp/$lib/libdmf.so
  DMF_LIB=$L timeout -k 10 400 python3 bench.py --steps 300 --no-secondary --cpu-frames 0 --pmc-dir $O/pmc_$lib > $O/bench_$lib.json 2> $O/bench_$lib.err || { echo "BENCHFAIL $lib"; tail -5 $O/bench_$lib.err; exit 4; }
  python3 tools/show_bench.py $O/bench_$lib.json | head -3
done
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_pipeline.py tests/test_gpu_parity.py tests/test_gpu_configs.py -k "fuse or long or pipelined or timed or guard or config or shard or anchor" > $O/tests.log 2>&1 || { echo FAIL tests; tail -20 $O/tests.log; exit 5; }
tail -2 $O/tests.log
echo ALLOK
