# Round-3 evidence after pipelining: default bench line (live PMC), a kernel
# trace of the pipelined bench with its timeline split, and the other single-GPU configs.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r03c
mkdir -p "$OUT"
timeout -k 10 400 python3 bench.py > "$OUT/bench_default.json" 2> "$OUT/bench_default.err" || { echo BENCHFAIL; tail "$OUT/bench_default.err"; exit 1; }
python3 tools/show_bench.py "$OUT/bench_default.json" || true
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kt" -o run -- python3 bench.py --steps 60 --warmup 3 --cpu-frames 0 --cpu-reverse-poses 0 --pmc off --no-secondary --serial-ref off > "$OUT/bench_kt.json" 2> "$OUT/bench_kt.err" || { echo KTFAIL; tail "$OUT/bench_kt.err"; exit 2; }
python3 tools/kt_timeline.py "$OUT/kt" 5 > "$OUT/timeline.txt" && cat "$OUT/timeline.txt"
timeout -k 10 300 python3 bench.py --grid 256 --poses-per-gpu 64 --cpu-frames 8 --no-secondary > "$OUT/config2.json" 2> "$OUT/config2.err" || { echo FAIL2; tail "$OUT/config2.err"; exit 3; }
timeout -k 10 300 python3 bench.py --poses-per-gpu 1024 --steps 12 --warmup 2 --cpu-frames 0 --no-secondary > "$OUT/anchor.json" 2> "$OUT/anchor.err" || { echo FAILA; tail "$OUT/anchor.err"; exit 4; }
timeout -k 10 400 python3 bench.py --image 1280x720 --grid 512 --poses-per-gpu 256 --steps 16 --warmup 2 --cpu-frames 2 --no-secondary > "$OUT/config3.json" 2> "$OUT/config3.err" || { echo FAIL3; tail "$OUT/config3.err"; exit 5; }
timeout -k 10 500 python3 bench.py --grid 1024 --poses-per-gpu 256 --image 1280x720 --steps 10 --warmup 2 --cpu-frames 0 --no-secondary > "$OUT/config5shard.json" 2> "$OUT/config5shard.err" || { echo FAIL5; tail "$OUT/config5shard.err"; exit 6; }
for f in config2 anchor config3 config5shard; do python3 -c "import json;d=json.load(open('$OUT/$f.json'));r=d['roofline'];print('$f', d['value'], d['ms_per_step'], r['frac'], r.get('serial_call_ms'), r.get('serial_call_frac'), r.get('measured_frac'))"; done
echo ALLOK
