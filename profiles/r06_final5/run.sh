#!/bin/bash
# Round 6 closing evidence: the GPU suite, smoke, the default bench line with its PMC child,
# the rocprofv3 trace + PMC passes (profile_round.sh), and the other single-GPU BASELINE
# workloads (config 2 twice: the 0.60 bar of VERDICT r5 #4).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
T=${TAG:-r06_final}
O=gpurun_out/$T
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo FAIL tests; tail -30 $O/gpu_tests.log; exit 4; }
tail -2 $O/gpu_tests.log
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { echo FAIL smoke; tail -20 $O/smoke.log; exit 5; }
tail -1 $O/smoke.log
timeout -k 10 400 python3 bench.py --pmc-dir $O/pmc_child > $O/bench_default.json 2> $O/bench_default.err || { echo BENCHFAIL; tail -20 $O/bench_default.err; exit 1; }
python3 tools/show_bench.py $O/bench_default.json | head -8
bash tools/profile_round.sh $T > $O/profile.log 2>&1 || { echo PROFFAIL; tail -5 $O/profile.log; exit 2; }
for cfg in "config2 --grid 256 --poses-per-gpu 64 --steps 400" "config2b --grid 256 --poses-per-gpu 64 --steps 400" "config3 --image 1280x720 --grid 512 --poses-per-gpu 256 --steps 12 --warmup 2" "anchor --grid 512 --poses-per-gpu 1024 --steps 12 --warmup 2" "config5shard --image 1280x720 --grid 1024 --poses-per-gpu 256 --steps 12 --warmup 2"; do
  set -- $cfg; name=$1; shift
  timeout -k 10 500 python3 bench.py "$@" --cpu-frames 0 --no-secondary --pmc off > $O/$name.json 2> $O/$name.err || { echo "FAIL $name"; tail -5 $O/$name.err; exit 3; }
  python3 tools/show_bench.py $O/$name.json | head -1
done
echo ALLOK
