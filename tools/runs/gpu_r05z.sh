#!/bin/bash
# Round 5: config 2 pipelined with phase F's queue tail split (DMF_KNOB_TAIL_SPLIT 1 / 2) and a
# smaller part cap (DMF_KNOB_PART_MAX 49152) vs the default, alternating, three repetitions.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r05z
mkdir -p $O
for rep in 1 2 3; do
  for kn in none tail_split=1 tail_split=2 part_max=49152; do
    K=""; [ $kn != none ] && K="--knob $kn"
    timeout -k 10 200 python3 tools/exp_fuse.py --grid 256 --poses 64 --calls 200 --modes pipelined $K > $O/c2_${kn}_$rep.json 2> /dev/null || { echo "FAIL $kn"; exit 3; }
    python3 -c "import json; c=json.load(open('$O/c2_${kn}_$rep.json')); print('$kn', round(c['pipelined_ms'],4), c['digest']=='605646542483b87f')"
  done
done
echo ALLOK
