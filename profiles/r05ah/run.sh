#!/bin/bash
# Round 5 (after the pass A / B instruction cuts): span re-sweep, config 2 (default 32) and the
# headline (default 64), alternating, three repetitions.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r05ah
mkdir -p $O
for rep in 1 2 3; do
  for sp in 0 24 48; do
    timeout -k 10 200 python3 tools/exp_fuse.py --grid 256 --poses 64 --calls 200 --modes pipelined --knob span=$sp > $O/c2_s${sp}_$rep.json 2> /dev/null || { echo "FAIL c2 $sp"; exit 3; }
    python3 -c "import json; c=json.load(open('$O/c2_s${sp}_$rep.json')); print('c2 span $sp', round(c['pipelined_ms'],4), c['digest']=='605646542483b87f')"
  done
  for sp in 0 32 48; do
    timeout -k 10 200 python3 tools/exp_fuse.py --calls 80 --modes pipelined --knob span=$sp > $O/c4_s${sp}_$rep.json 2> /dev/null || { echo "FAIL c4 $sp"; exit 3; }
    python3 -c "import json; c=json.load(open('$O/c4_s${sp}_$rep.json')); print('c4 span $sp', round(c['pipelined_ms'],4), c['digest']=='36708f70245952ff')"
  done
done
echo ALLOK
