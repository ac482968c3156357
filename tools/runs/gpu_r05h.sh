#!/bin/bash
# Round 5: the pass-B layout guard test alone first (it walks a corrupted layout on purpose),
# then the full GPU suite, the headline bench and config 2.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r05h
mkdir -p $O
timeout -k 10 120 python -u -m pytest tests/test_gpu_pipeline.py -m gpu -x -v --timeout 100 --timeout-method thread -k "layout_guard" > $O/guard.log 2>&1 || { echo GUARDFAIL; tail -30 $O/guard.log; exit 1; }
tail -2 $O/guard.log
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo TESTFAIL; tail -40 $O/gpu_tests.log; exit 2; }
tail -2 $O/gpu_tests.log
timeout -k 10 300 python bench.py --grid 256 --poses-per-gpu 64 --pmc off --cpu-frames 0 --no-secondary > $O/config2.json 2> $O/config2.err || { echo CFG2FAIL; tail -20 $O/config2.err; exit 3; }
python tools/show_bench.py $O/config2.json | head -2
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || { echo BENCHFAIL; tail -30 $O/bench.err; exit 4; }
python tools/show_bench.py $O/bench.json
echo ALLOK
