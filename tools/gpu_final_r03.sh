# Round-3 closing run: GPU suite + smoke + default bench line, then config 2's line (pipelined).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/gpu_check.sh || exit 1
timeout -k 10 300 python3 bench.py --grid 256 --poses-per-gpu 64 --cpu-frames 8 --no-secondary > gpurun_out/config2_final.json 2> gpurun_out/config2_final.err || { echo FAIL2; tail gpurun_out/config2_final.err; exit 2; }
python3 tools/show_bench.py gpurun_out/config2_final.json
echo FINALOK
