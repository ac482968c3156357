#!/bin/bash
# Round 6: pass B's lane utilisation (DMF_EXP_STATS build: wave iterations of the brick replay
# loop and the lanes active in them) beside phase F's.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r06l
mkdir -p $O
B=depth-map-fusion-utils_amd
DMF_LIB=$B/build_exp/stats/libdmf.so timeout -k 10 300 python3 bench.py --steps 20 --no-secondary --cpu-frames 0 --pmc off --serial-ref off > $O/bench_stats.json 2> $O/bench_stats.err || { echo STATSFAIL; tail -5 $O/bench_stats.err; exit 6; }
python3 -c "import json; b=json.load(open('$O/bench_stats.json')); print(json.dumps(b['fuse_diagnostics']))"
echo ALLOK
