# Optional GPU test selection ($TESTS, pytest -k $TESTK), then alternating fusion bench
# lines of the fusion variants $VARIANTS (DMF_FUSE_VARIANT) on the same box, $ROUNDS rounds.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/var
if [ -n "$TESTS" ]; then
  timeout -k 10 ${TEST_TIMEOUT:-900} python -u -m pytest $TESTS -x -v --timeout 300 --timeout-method thread ${TESTK:+-k "$TESTK"} > gpurun_out/var/tests.log 2>&1 || { echo TESTFAIL; tail -40 gpurun_out/var/tests.log; exit 1; }
  tail -3 gpurun_out/var/tests.log
fi
for i in $(seq 1 ${ROUNDS:-3}); do
  for V in ${VARIANTS:-0 53}; do
    DMF_FUSE_VARIANT=$V timeout -k 10 200 python3 bench.py --steps ${STEPS:-300} --warmup 3 --pmc off --cpu-frames 0 --cpu-reverse-poses 0 --no-secondary ${BENCHARGS} > gpurun_out/var/v$V.$i.json 2> gpurun_out/var/v$V.$i.err || { echo BENCHFAIL $V; tail gpurun_out/var/v$V.$i.err; exit 2; }
    python3 -c "import json; d=json.load(open('gpurun_out/var/v$V.$i.json')); print('v$V', '%.3f ms'%d['roofline']['kernel_ms'], '%.4e'%d['value'], 'frac %.3f'%d['roofline']['frac'], d['roofline']['kernel'])"
  done
done
echo ALLOK
