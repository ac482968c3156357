# Round evidence: GPU suite, smoke, default bench line, then the other single-GPU BASELINE
# configurations and the config-4 strong-scaling anchor (all 1024 poses on one GPU).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/cfg
bash tools/gpu_check.sh || exit 1
# timed steps sized to ~1 s of work each (the counter clear overlaps from the third step on)
for c in "anchor --steps 12 --poses-per-gpu 1024" "config2 --steps 300 --grid 256 --poses-per-gpu 64" "config3 --steps 20 --grid 512 --poses-per-gpu 256 --image 1280x720" "config5shard --steps 8 --grid 1024 --poses-per-gpu 256 --image 1280x720" "config5grid32 --steps 60 --grid 1024 --poses-per-gpu 32 --image 1280x720"; do
  set -- $c; name=$1; shift
  timeout -k 10 400 python bench.py --warmup 2 "$@" > gpurun_out/cfg/$name.json 2> gpurun_out/cfg/$name.err || { echo CFGFAIL $name; tail -5 gpurun_out/cfg/$name.err; exit 2; }
  python3 -c "import json; d=json.load(open('gpurun_out/cfg/$name.json')); print('$name', d['config']['workload'][:40], '%.3e'%d['value'], '%.2f ms'%d['roofline']['kernel_ms'], 'frac %.3f'%d['roofline']['frac'], 'traffic', d['roofline']['traffic'])"
done
echo ROUNDOK
