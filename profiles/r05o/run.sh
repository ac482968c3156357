#!/bin/bash
# Round 5: the reverse parity over distance caps on the shipped (clipped-cube) march, then
# config 5's 1024^3 shard with the default 55 % fusion budget (one pose batch expected).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r05o
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_parity.py -k "reverse" > $O/tests.log 2>&1 || { echo FAIL tests; tail -20 $O/tests.log; exit 4; }
tail -2 $O/tests.log
timeout -k 10 600 python3 bench.py --image 1280x720 --grid 1024 --poses-per-gpu 256 --steps 12 --warmup 2 --cpu-frames 0 --no-secondary --pmc off > $O/config5shard.json 2> $O/config5shard.err || { echo FAIL c5; tail -20 $O/config5shard.err; exit 5; }
python3 -c "import json; d=json.load(open('$O/config5shard.json')); print(d['ms_per_step'], d['roofline']['frac'], d['fuse_plan'], d['digest_match'])"
echo ALLOK
