# Round 3 check: full GPU suite, fusion A/B (20-B vs 24-B records), one bench line with the
# secondary kernels (reverse visibility, forward march) for their timings.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r03a
TESTS="tests -m gpu" TEST_TIMEOUT=900 ROUNDS=3 VARIANTS="0 53" bash tools/gpu_var_ab.sh || exit 1
timeout -k 10 300 python3 bench.py --steps 300 --warmup 3 --pmc off --cpu-frames 0 --cpu-reverse-poses 0 > gpurun_out/r03a/bench.json 2> gpurun_out/r03a/bench.err || { echo BENCHFAIL; tail gpurun_out/r03a/bench.err; exit 2; }
python3 - <<'PY'
import json
d = json.load(open("gpurun_out/r03a/bench.json"))
s = d["secondary"]
print("fusion", "%.3f ms" % d["roofline"]["kernel_ms"], "%.4e" % d["value"], "frac %.3f" % d["roofline"]["frac"])
print("reverse ms/batch %.3f" % s["reverse_ray_trace_fast"]["ms_per_batch"], "samples/s %.3e" % s["reverse_ray_trace_fast"]["march_samples_per_s"])
print("forward ms/batch %.3f" % s["forward_first_hits"]["ms_per_batch"])
PY
echo R03A_OK
