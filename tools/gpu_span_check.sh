# GPU suite after the A/B span rule, then the config 2 line.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/cfg
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo TESTFAIL; tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
timeout -k 10 400 python bench.py --warmup 2 --steps 300 --grid 256 --poses-per-gpu 64 > gpurun_out/cfg/config2.json 2> gpurun_out/cfg/config2.err || { echo CFGFAIL; tail -5 gpurun_out/cfg/config2.err; exit 2; }
python3 -c "import json; d=json.load(open('gpurun_out/cfg/config2.json')); print('config2', '%.3e'%d['value'], '%.3f ms'%d['roofline']['kernel_ms'], 'frac %.3f'%d['roofline']['frac'])"
echo CHECKOK
