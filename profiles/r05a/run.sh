#!/bin/bash
# Round 5, first GPU pass: host CPU share probe, the new GPU tests, the full GPU suite, smoke,
# the default bench line, and the self-launched 2-rank gloo rehearsal (bench.py --gpus 2, no wrapper).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r05a
mkdir -p $O
{ echo "nproc $(nproc)"; cat /sys/fs/cgroup/cpu.max 2>&1; python -c 'import os; print("affinity", len(os.sched_getaffinity(0)), "omp", os.environ.get("OMP_NUM_THREADS"))'; lscpu | head -20; } > $O/host.txt 2>&1
timeout -k 10 400 python -u -m pytest tests/test_gpu_pipeline.py -m gpu -x -v --timeout 240 --timeout-method thread -k "layout_guard" > $O/new_tests.log 2>&1 || { echo NEWTESTFAIL; tail -40 $O/new_tests.log; exit 1; }
tail -3 $O/new_tests.log
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo TESTFAIL; tail -40 $O/gpu_tests.log; exit 1; }
tail -3 $O/gpu_tests.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SMOKEFAIL; tail -20 $O/smoke.log; exit 2; }
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || { echo BENCHFAIL; tail -30 $O/bench.err; exit 3; }
python tools/show_bench.py $O/bench.json 2>/dev/null | head -40 || true
DMF_BENCH_BACKEND=gloo timeout -k 10 400 python bench.py --gpus 2 --steps 20 --warmup 3 --pmc off --no-secondary --cpu-frames 0 --serial-ref off > $O/bench_n2_gloo.json 2> $O/bench_n2_gloo.err || { echo DISTFAIL; tail -30 $O/bench_n2_gloo.err; exit 4; }
cat $O/bench_n2_gloo.json | head -c 1500
echo ALLOK
