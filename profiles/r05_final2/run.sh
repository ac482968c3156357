#!/bin/bash
# Round 5 final evidence (after the 96-VGPR pass B and the 7-wave reverse march): rocprofv3 kernel trace + PMC passes of the default bench (profile_round.sh),
# the default bench line with its PMC kept, and the other single-GPU BASELINE workloads.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r05_final2
mkdir -p $O
timeout -k 10 400 python bench.py --pmc-dir $O/pmc_child > $O/bench_default.json 2> $O/bench_default.err || { echo BENCHFAIL; tail -20 $O/bench_default.err; exit 1; }
python tools/show_bench.py $O/bench_default.json | head -4
bash tools/profile_round.sh r05_final2 || { echo PROFFAIL; exit 2; }
for cfg in "config2 --grid 256 --poses-per-gpu 64 --steps 400" "config3 --image 1280x720 --grid 512 --poses-per-gpu 256 --steps 12 --warmup 2" "anchor --grid 512 --poses-per-gpu 1024 --steps 12 --warmup 2" "config5shard --image 1280x720 --grid 1024 --poses-per-gpu 256 --steps 12 --warmup 2"; do
  set -- $cfg; name=$1; shift
  timeout -k 10 500 python3 bench.py "$@" --cpu-frames 0 --no-secondary --pmc off > $O/$name.json 2> $O/$name.err || { echo "FAIL $name"; tail -5 $O/$name.err; exit 3; }
  python3 tools/show_bench.py $O/$name.json | head -2
done
echo ALLOK
