# A/B of env settings on the headline bench (pipelined default): ENVS="A=1,B=2 A=0 ..." (comma =
# several vars in one setting), REPS rounds; then optional kernel-trace timeline of KT_ENV.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/envab
mkdir -p "$OUT"
if [ -n "$TESTS" ]; then
  timeout -k 10 500 python -u -m pytest $TESTS -x -q --timeout 180 --timeout-method thread > "$OUT/tests.log" 2>&1 || { echo TESTFAIL; tail -30 "$OUT/tests.log"; exit 1; }
  tail -1 "$OUT/tests.log"
fi
i=0
for r in $(seq ${REPS:-2}); do
  for e in $ENVS; do
    i=$((i+1))
    env $(echo $e | tr ',' ' ') timeout -k 10 200 python bench.py --steps ${STEPS:-400} --no-secondary --pmc off --cpu-frames 0 --serial-ref off ${BENCH_ARGS:-} > "$OUT/b$i.json" 2> "$OUT/b$i.err" || { echo BENCHFAIL $e; tail "$OUT/b$i.err"; exit 2; }
    python -c "import json;d=json.load(open('$OUT/b$i.json'));r=d['roofline'];print('$e', round(d['value']/1e12,4), round(d['ms_per_step'],4), round(r['frac'],4), d['logodds_digest'])"
  done
done
if [ -n "$KT_ENV" ]; then
  env $(echo $KT_ENV | tr ',' ' ') timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kt" -o run -- python3 bench.py --steps 60 --warmup 3 --cpu-frames 0 --cpu-reverse-poses 0 --pmc off --no-secondary --serial-ref off ${BENCH_ARGS:-} > "$OUT/bench_kt.json" 2> "$OUT/bench_kt.err" || { echo KTFAIL; tail "$OUT/bench_kt.err"; exit 3; }
  python3 tools/kt_timeline.py "$OUT/kt" 5
fi
echo ALLOK
