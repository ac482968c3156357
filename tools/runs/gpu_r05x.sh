#!/bin/bash
# Round 5: the bench's own pipelined step (phase event set) with the layout / pass B on the
# volume's stream vs the staging-stream pass B (strm0), alternating; headline and config 2;
# then the pipeline tests.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r05x
mkdir -p $O
B=depth-map-fusion-utils_amd
for rep in 1 2 3; do
  for lib in product strm0; do
    L=$B/build/libdmf.so; [ $lib != product ] && L=$B/build_exp/$lib/libdmf.so
    DMF_LIB=$L timeout -k 10 300 python3 bench.py --steps 400 --warmup 5 --no-secondary --pmc off --cpu-frames 0 --serial-ref off > $O/c4_${lib}_$rep.json 2> $O/c4_${lib}_$rep.err || { echo "FAIL c4 $lib"; tail -5 $O/c4_${lib}_$rep.err; exit 3; }
    DMF_LIB=$L timeout -k 10 300 python3 bench.py --grid 256 --poses-per-gpu 64 --steps 1000 --warmup 5 --no-secondary --pmc off --cpu-frames 0 --serial-ref off > $O/c2_${lib}_$rep.json 2> $O/c2_${lib}_$rep.err || { echo "FAIL c2 $lib"; tail -5 $O/c2_${lib}_$rep.err; exit 3; }
    python3 -c "import json; b=json.load(open('$O/c4_${lib}_$rep.json')); c=json.load(open('$O/c2_${lib}_$rep.json')); print('$lib', round(b['ms_per_step'],4), round(b['roofline']['frac'],4), b['digest_match'], round(c['ms_per_step'],4), round(c['roofline']['frac'],4), c['digest_match'])"
  done
done
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_pipeline.py tests/test_gpu_boundary.py > $O/tests.log 2>&1 || { echo FAIL tests; tail -20 $O/tests.log; exit 4; }
tail -2 $O/tests.log
echo ALLOK
