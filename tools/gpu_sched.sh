# Bench lines after a schedule change: default workload, config 5's shard and config 2.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/sched
timeout -k 10 300 python3 bench.py --pmc off --cpu-frames 0 --cpu-reverse-poses 0 --no-secondary > gpurun_out/sched/default.json 2> gpurun_out/sched/default.err || { echo BENCHFAIL default; tail gpurun_out/sched/default.err; exit 2; }
timeout -k 10 300 python3 bench.py --steps 60 --pmc off --cpu-frames 0 --cpu-reverse-poses 0 --no-secondary --grid 1024 --image 1280x720 --poses-per-gpu 32 > gpurun_out/sched/c5.json 2> gpurun_out/sched/c5.err || { echo BENCHFAIL c5; tail gpurun_out/sched/c5.err; exit 2; }
timeout -k 10 300 python3 bench.py --steps 300 --pmc off --cpu-frames 0 --cpu-reverse-poses 0 --no-secondary --grid 256 --poses-per-gpu 64 > gpurun_out/sched/c2.json 2> gpurun_out/sched/c2.err || { echo BENCHFAIL c2; tail gpurun_out/sched/c2.err; exit 2; }
for n in default c5 c2; do python3 -c "import json; d=json.load(open('gpurun_out/sched/$n.json')); print('$n', '%.3e'%d['value'], 'step %.3f'%d['ms_per_step'], 'fuse %.3f'%d['roofline']['kernel_ms'], 'frac %.3f'%d['roofline']['frac'], {k:round(v,3) for k,v in d['step_breakdown_ms'].items() if isinstance(v,float)}, d['roofline']['kernel'])"; done
echo ALLOK
