#!/bin/bash
# Round 5: pass A/B workgroup span (DMF_KNOB_SPAN, 8x8 packets per workgroup) at config 2
# (default 32) and the headline (default 64), pipelined calls.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r05u
mkdir -p $O
for rep in 1 2; do
  for sp in 0 16 64 128; do
    timeout -k 10 200 python3 tools/exp_fuse.py --grid 256 --poses 64 --calls 150 --modes pipelined --knob span=$sp > $O/c2_s${sp}_$rep.json 2> /dev/null || { echo "FAIL c2 $sp"; exit 3; }
    python3 -c "import json; c=json.load(open('$O/c2_s${sp}_$rep.json')); print('c2 span $sp', round(c['pipelined_ms'],4), c['digest']=='605646542483b87f')"
  done
  for sp in 0 32 128; do
    timeout -k 10 200 python3 tools/exp_fuse.py --calls 60 --modes pipelined --knob span=$sp > $O/c4_s${sp}_$rep.json 2> /dev/null || { echo "FAIL c4 $sp"; exit 3; }
    python3 -c "import json; c=json.load(open('$O/c4_s${sp}_$rep.json')); print('c4 span $sp', round(c['pipelined_ms'],4), c['digest']=='36708f70245952ff')"
  done
done
echo ALLOK
