# kernel traces of the brick pipeline at 256^3 (64 frames) and 1024^3 (32 frames)
set -o pipefail
mkdir -p gpurun_out/grid
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/grid/kt256 -o run -- python3 bench.py --grid 256 --poses-per-gpu 64 --steps 2 --warmup 1 --cpu-frames 0 --no-secondary > gpurun_out/grid/kt256.json 2> gpurun_out/grid/kt256.err || { echo FAIL256; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/grid/kt1024 -o run -- python3 bench.py --grid 1024 --poses-per-gpu 32 --steps 2 --warmup 1 --cpu-frames 0 --no-secondary > gpurun_out/grid/kt1024.json 2> gpurun_out/grid/kt1024.err || { echo FAIL1024; exit 2; }
echo ALLOK
