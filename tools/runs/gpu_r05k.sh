#!/bin/bash
# Round 5: kernel trace of the headline's pipelined calls (per-call timeline).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r05k
mkdir -p $O
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_c4 -o run -- python3 tools/exp_fuse.py --grid 512 --poses 128 --calls 30 --modes pipelined > $O/c4.json 2> $O/kt_c4.err || { echo KTFAIL; exit 4; }
cat $O/c4.json
echo ALLOK
