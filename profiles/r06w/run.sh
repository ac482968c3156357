#!/bin/bash
# Round 6: the headline call cut into two or four super-batches (DMF_KNOB_SUPER_POSES 64 / 32: pass A
# of the second half beside the first half's pass B and phase F) vs one (128 poses), pipelined and
# serial; alternating, two repetitions.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r06w
mkdir -p $O
for rep in 1 2; do
  for v in "default:" "sp64:super_poses=64" "sp32:super_poses=32"; do
    tag=${v%%:*}; kn=${v#*:}; args=""; [ -n "$kn" ] && args="--knob $kn"
    timeout -k 10 200 python3 tools/exp_fuse.py --tag $tag --calls 60 $args > $O/c4_${tag}_$rep.json 2> $O/c4_${tag}_$rep.err || { echo "FAIL $tag"; tail -5 $O/c4_${tag}_$rep.err; exit 3; }
    python3 -c "import json; c=json.load(open('$O/c4_${tag}_$rep.json')); print('$tag', round(c['serial_ms'],4), round(c['pipelined_ms'],4), c['digest']=='36708f70245952ff')"
  done
done
echo ALLOK
