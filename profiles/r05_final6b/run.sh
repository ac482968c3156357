#!/bin/bash
# Round 5: the closing build's default bench line on a second box (box-to-box spread of the
# headline; profiles/r05_final6 came from a box whose phase F ran 4.00 ms).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r05_final6b
mkdir -p $O
timeout -k 10 400 python3 bench.py --pmc-dir $O/pmc_child > $O/bench_default.json 2> $O/bench_default.err || { echo BENCHFAIL; tail -20 $O/bench_default.err; exit 1; }
python3 tools/show_bench.py $O/bench_default.json | head -3
timeout -k 10 500 python3 bench.py --grid 256 --poses-per-gpu 64 --steps 400 --cpu-frames 0 --no-secondary --pmc off > $O/config2.json 2> $O/config2.err || { echo "FAIL config2"; tail -5 $O/config2.err; exit 3; }
python3 tools/show_bench.py $O/config2.json | head -1
echo ALLOK
