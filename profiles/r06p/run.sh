#!/bin/bash
# Round 6: where config 2's pipelined step goes (kernel-trace timeline, 256^3, 64 poses) beside
# the headline's, with the closing build.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r06p
mkdir -p $O
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/kt_c2 -o run -- python3 tools/exp_fuse.py --grid 256 --poses 64 --calls 100 --modes pipelined > $O/kt_c2.json 2> $O/kt_c2.err || { echo KTFAIL; tail -5 $O/kt_c2.err; exit 1; }
python3 tools/kt_timeline.py $O/kt_c2 20 > $O/timeline_c2.txt 2>&1; tail -25 $O/timeline_c2.txt
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/kt_c4 -o run -- python3 tools/exp_fuse.py --calls 40 --modes pipelined > $O/kt_c4.json 2> $O/kt_c4.err || { echo KTFAIL; exit 2; }
python3 tools/kt_timeline.py $O/kt_c4 10 > $O/timeline_c4.txt 2>&1; tail -25 $O/timeline_c4.txt
echo ALLOK
