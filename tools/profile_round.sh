#!/bin/bash
# Collect the rocprofv3 evidence for one round (run on the GPU box via gpurun):
#   1) kernel trace + stats of the default bench command,
#   2) separate PMC passes (never combined with sys/runtime traces):
#      FETCH_SIZE | WRITE_SIZE | TCC_EA0_ATOMIC_sum,TCC_HIT_sum,TCC_MISS_sum | SQ_* busy/wait
# then summarise into profiles/<tag>/ and profiles/pmc_fuse_summary.json.
set -o pipefail
TAG=${1:-r01}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/prof_$TAG
mkdir -p "$OUT"
BENCH="python3 bench.py --steps 20 --warmup 2 --cpu-frames 0 --cpu-reverse-poses 0 --pmc off ${BENCHARGS}"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kt" -o run -- $BENCH > "$OUT/bench_kt.json" 2> "$OUT/bench_kt.err" || exit 1
i=0
for pmc in "FETCH_SIZE" "WRITE_SIZE" "TCC_EA0_ATOMIC_sum TCC_HIT_sum TCC_MISS_sum" "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS" "SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -k 10 400 rocprofv3 --pmc $pmc --output-format csv -d "$OUT/pmc$i" -o run -- python3 bench.py --steps 1 --warmup 0 --cpu-frames 0 --no-secondary --pmc off --serial-ref off ${BENCHARGS} > "$OUT/pmc$i.json" 2> "$OUT/pmc$i.err" || exit 2
done
# extra counter groups (";"-separated in $EXTRA_PMC); counters the box does not list are dropped
if [ -n "$EXTRA_PMC" ]; then
  timeout -k 10 120 rocprofv3 -L > "$OUT/counters.txt" 2>&1 || true
  IFS=';' read -ra GROUPS_X <<< "$EXTRA_PMC"
  for grp in "${GROUPS_X[@]}"; do
    keep=""
    for c in $grp; do
      base=${c%_sum}
      if grep -qw -- "$base" "$OUT/counters.txt"; then keep="$keep $c"; else echo "counter $c not listed: dropped"; fi
    done
    [ -z "$keep" ] && continue
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --pmc $keep --output-format csv -d "$OUT/pmc$i" -o run -- python3 bench.py --steps 1 --warmup 0 --cpu-frames 0 --no-secondary --pmc off --serial-ref off ${BENCHARGS} > "$OUT/pmc$i.json" 2> "$OUT/pmc$i.err" || exit 2
  done
fi
python3 tools/pmc_summary.py "$OUT" "profiles/$TAG" || exit 3
echo "profile $TAG collected"
