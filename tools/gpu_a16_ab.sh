# Pass A with 16-bit histogram counts (DMF_BK_A16): parity (pipeline tests and
# the brick tests at the default), A/B bench lines, kernel-trace timeline of the default.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/a16
mkdir -p "$OUT"
timeout -k 10 500 python -u -m pytest tests/test_gpu_pipeline.py tests/test_gpu_parity.py -k "pipelined or brick_path or multi_batch or full_size or edge" -x -q --timeout 180 --timeout-method thread > "$OUT/tests.log" 2>&1 || { echo TESTFAIL; tail -30 "$OUT/tests.log"; exit 1; }
tail -2 "$OUT/tests.log"
for m in 1 0 1 0; do
  DMF_BK_A16=$m timeout -k 10 200 python bench.py --steps 400 --no-secondary --pmc off --cpu-frames 0 --serial-ref off ${BENCH_ARGS:-} > "$OUT/b$m.json" 2> "$OUT/b$m.err" || { echo BENCHFAIL; tail "$OUT/b$m.err"; exit 2; }
  python -c "import json;d=json.load(open('$OUT/b$m.json'));r=d['roofline'];print('a16=$m', round(d['value']/1e12,4), round(d['ms_per_step'],4), round(r['frac'],4), d['logodds_digest'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kt" -o run -- python3 bench.py --steps 60 --warmup 3 --cpu-frames 0 --cpu-reverse-poses 0 --pmc off --no-secondary --serial-ref off ${BENCH_ARGS:-} > "$OUT/bench_kt.json" 2> "$OUT/bench_kt.err" || { echo KTFAIL; tail "$OUT/bench_kt.err"; exit 3; }
python3 tools/kt_timeline.py "$OUT/kt" 5
echo ALLOK
