# Round-4 first run: the GPU suite (incl. the new timed-mode, edge-case and golden-digest
# tests), smoke, the default bench line with its PMC / kernel-trace children, config 2.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/${TAG:-r04a}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?
tail -40 $O/gpu_tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || { echo "TESTS ABORTED rc=$rc"; exit 1; }
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SMOKEFAIL; tail -20 $O/smoke.log; exit 2; }
timeout -k 10 400 python bench.py --pmc-dir $O/pmc > $O/bench.json 2> $O/bench.err || { echo BENCHFAIL; tail -20 $O/bench.err; exit 3; }
python3 tools/show_bench.py $O/bench.json || true
timeout -k 10 300 python3 bench.py --grid 256 --poses-per-gpu 64 --cpu-frames 8 --no-secondary > $O/config2.json 2> $O/config2.err || { echo FAIL2; tail $O/config2.err; exit 4; }
python3 tools/show_bench.py $O/config2.json
echo "TESTRC $rc"
echo ALLOK
