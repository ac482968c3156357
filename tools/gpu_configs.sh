# bench lines for the other single-GPU BASELINE configs: 2 (640x480, 256^3, 64 poses) and
# 3 (1280x720, 512^3, 256 poses), with the CPU oracle sample
set -o pipefail
mkdir -p gpurun_out/configs
timeout -k 10 400 python bench.py --grid 256 --poses-per-gpu 64 --cpu-frames 8 > gpurun_out/configs/config2.json 2> gpurun_out/configs/config2.err || { echo FAIL2; tail gpurun_out/configs/config2.err; exit 1; }
timeout -k 10 600 python bench.py --image 1280x720 --grid 512 --poses-per-gpu 256 --steps 3 --warmup 1 --cpu-frames 2 > gpurun_out/configs/config3.json 2> gpurun_out/configs/config3.err || { echo FAIL3; tail gpurun_out/configs/config3.err; exit 2; }
echo ALLOK
