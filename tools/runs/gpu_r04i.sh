# Round-4 run i: the long-ray test (pass B's walk fallback), then bench lines for the other
# single-GPU BASELINE workloads: config 3 (1280x720, 512^3, 256 poses), the config-4 anchor
# (1024 poses on one GPU) and config 5's per-GPU shard (1280x720, 1024^3, 256 poses).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/${TAG:-r04i}
mkdir -p $O
export TMPDIR=/tmp
true
true
for cfg in "config3 --image 1280x720 --grid 512 --poses-per-gpu 256" "anchor --grid 512 --poses-per-gpu 1024" "config5shard --image 1280x720 --grid 1024 --poses-per-gpu 256"; do
  set -- $cfg; name=$1; shift
  timeout -k 10 500 python3 bench.py "$@" --steps 12 --warmup 2 --cpu-frames 0 --no-secondary --pmc off > $O/$name.json 2> $O/$name.err || { echo "FAIL $name"; tail -5 $O/$name.err; exit 2; }
  python3 tools/show_bench.py $O/$name.json | head -2
done
echo R04IOK
