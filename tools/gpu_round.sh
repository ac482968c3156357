# Round evidence on one GPU box: full GPU test suite, smoke, default bench line, then the
# rocprofv3 kernel trace + PMC passes of tools/profile_round.sh (tag $1).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo TESTFAIL; tail -30 gpurun_out/gpu_tests.log; exit 1; }
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo SMOKEFAIL; tail -20 gpurun_out/smoke.log; exit 2; }
timeout -k 10 400 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo BENCHFAIL; tail -20 gpurun_out/bench.err; exit 3; }
bash tools/profile_round.sh "${1:-r01}" > gpurun_out/profile.log 2>&1 || { echo PROFFAIL; tail -20 gpurun_out/profile.log; exit 4; }
echo ALLOK
