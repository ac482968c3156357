#!/bin/bash
# Round 5: reverseRayTraceFast with the empty cube not clipped to the volume (a jump may land
# past the volume's faces: "left the volume" at once) and the brick distance cap
# (DMF_KNOB_BDIST_CAP 63 / 127 / 255) vs the clipped cube (experiment build revclip); then the
# reverse parity tests and the bench-size march digests.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r05m
mkdir -p $O
B=depth-map-fusion-utils_amd
DMF_LIB=$B/build_exp/revclip/libdmf.so timeout -k 10 300 python3 tools/exp_reverse.py 0,0 0,255 > $O/clip.json 2> $O/clip.err || { echo FAIL clip; tail -5 $O/clip.err; exit 3; }
cat $O/clip.json
timeout -k 10 300 python3 tools/exp_reverse.py 0,0 0,127,255 > $O/ext.json 2> $O/ext.err || { echo FAIL ext; tail -5 $O/ext.err; exit 3; }
cat $O/ext.json
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_marches.py "tests/test_gpu_parity.py" -k "reverse or marches" > $O/tests.log 2>&1 || { echo FAIL tests; tail -20 $O/tests.log; exit 4; }
tail -3 $O/tests.log
echo ALLOK
