#!/bin/bash
# Round 6: config 2's part queue re-swept after this round's phase-F changes (pipelined calls):
# part cap 32768 / 49152 and the tail split at 1 / 2 / 4 x CUs vs the defaults (65535, no split
# when pipelined); alternating, two repetitions.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r06q
mkdir -p $O
for rep in 1 2; do
  for v in "default:" "pm32k:part_max=32768" "pm48k:part_max=49152" "ts1:tail_split=1" "ts2:tail_split=2" "ts4:tail_split=4"; do
    tag=${v%%:*}; kn=${v#*:}; args=""; [ -n "$kn" ] && args="--knob $kn"
    timeout -k 10 200 python3 tools/exp_fuse.py --tag $tag --grid 256 --poses 64 --calls 150 $args > $O/c2_${tag}_$rep.json 2> $O/c2_${tag}_$rep.err || { echo "FAIL $tag"; tail -5 $O/c2_${tag}_$rep.err; exit 3; }
    python3 -c "import json; c=json.load(open('$O/c2_${tag}_$rep.json')); print('$tag', round(c['serial_ms'],4), round(c['pipelined_ms'],4), c['digest']=='605646542483b87f')"
  done
done
echo ALLOK
