#!/bin/bash
# Round 6: phase F at issue priority 1 (fprio) vs the product in the bench's step (finalize and
# clear beside F, the next call's pass A beside F) and in fusion calls alone; alternating.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r06r
mkdir -p $O
B=depth-map-fusion-utils_amd
for rep in 1 2; do
  for lib in product fprio; do
    L=$B/build/libdmf.so; [ $lib != product ] && L=$B/build_exp/$lib/libdmf.so
    DMF_LIB=$L timeout -k 10 300 python3 bench.py --steps 400 --no-secondary --cpu-frames 0 --pmc off --serial-ref off > $O/bench_${lib}_$rep.json 2> $O/bench_${lib}_$rep.err || { echo "FAIL $lib"; tail -5 $O/bench_${lib}_$rep.err; exit 3; }
    DMF_LIB=$L timeout -k 10 200 python3 tools/exp_fuse.py --tag $lib --calls 60 --modes pipelined > $O/c4_${lib}_$rep.json 2> /dev/null || { echo "FAIL $lib"; exit 3; }
    python3 -c "import json; b=json.load(open('$O/bench_${lib}_$rep.json')); c=json.load(open('$O/c4_${lib}_$rep.json')); print('$lib', 'bench', round(b['ms_per_step'],4), b['digest_match'], 'fuse-only', round(c['pipelined_ms'],4), c['digest']=='36708f70245952ff')"
  done
done
echo ALLOK
