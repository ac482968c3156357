#!/bin/bash
# Round 5: span sweep at 512^3 (headline 640x480 x 128; config 3 1280x720 x 256 pipelined).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r05v
mkdir -p $O
for rep in 1 2; do
  for sp in 0 16 24 32 48; do
    timeout -k 10 200 python3 tools/exp_fuse.py --calls 60 --modes pipelined --knob span=$sp > $O/c4_s${sp}_$rep.json 2> /dev/null || { echo "FAIL c4 $sp"; exit 3; }
    python3 -c "import json; c=json.load(open('$O/c4_s${sp}_$rep.json')); print('c4 span $sp', round(c['pipelined_ms'],4), c['digest']=='36708f70245952ff')"
  done
done
for sp in 0 32; do
  timeout -k 10 300 python3 tools/exp_fuse.py --image 1280x720 --poses 256 --calls 12 --modes pipelined --knob span=$sp > $O/c3_s${sp}.json 2> $O/c3_s${sp}.err || { echo "FAIL c3 $sp"; tail -3 $O/c3_s${sp}.err; exit 3; }
  python3 -c "import json; c=json.load(open('$O/c3_s${sp}.json')); print('c3 span $sp', round(c['pipelined_ms'],4), c['digest'])"
done
echo ALLOK
