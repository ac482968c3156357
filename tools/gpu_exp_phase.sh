# Bench step with the merge / clear of step i deferred behind step i+1's phase-F event
# (default) vs right after step i's fusion (DMF_BENCH_PHASE=0), alternating on one box.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/exp_phase
mkdir -p $O
for k in 1 0 1 0; do
  i=$((i+1))
  DMF_BENCH_PHASE=$k timeout -k 10 300 python3 bench.py --steps 600 --no-secondary --pmc off --cpu-frames 0 --serial-ref off > $O/phase${k}_$i.json 2> $O/phase${k}_$i.err || { echo "FAIL $k"; tail -5 $O/phase${k}_$i.err; exit 1; }
  python3 -c "import json,sys; b=json.load(open('$O/phase${k}_$i.json')); print('phase $k', round(b['ms_per_step'],4), b['roofline']['frac'], b.get('digest_match'), b['step_breakdown_ms'] if 'step_breakdown_ms' in b else '')" 2>/dev/null || python3 tools/show_bench.py $O/phase${k}_$i.json | head -2
done
timeout -k 10 300 python3 bench.py --grid 256 --poses-per-gpu 64 --steps 1000 --no-secondary --pmc off --cpu-frames 0 --serial-ref off > $O/cfg2_phase1.json 2> $O/cfg2_phase1.err && python3 tools/show_bench.py $O/cfg2_phase1.json | head -1
DMF_BENCH_PHASE=0 timeout -k 10 300 python3 bench.py --grid 256 --poses-per-gpu 64 --steps 1000 --no-secondary --pmc off --cpu-frames 0 --serial-ref off > $O/cfg2_phase0.json 2> $O/cfg2_phase0.err && python3 tools/show_bench.py $O/cfg2_phase0.json | head -1
echo PHASEOK
