# reverseRayTraceFast kernel A/B ($REVS, DMF_REVERSE_KERNEL): parity tests, then the bench's
# secondary reverse line with live PMC (L2 hit rate, issue fraction).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/rev
export TMPDIR=/tmp
for K in ${REVS:-2}; do
  DMF_REVERSE_KERNEL=$K timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_reference_driver.py -m gpu -x -q --timeout 120 --timeout-method thread -k "${TESTK:-reverse or visib or raytracing or setcover or set_cover}" > gpurun_out/rev/tests$K.log 2>&1 || { echo TESTFAIL $K; tail -30 gpurun_out/rev/tests$K.log; exit 1; }
  tail -1 gpurun_out/rev/tests$K.log
  DMF_REVERSE_KERNEL=$K timeout -k 10 300 python3 bench.py --steps 3 --warmup 1 --cpu-frames 0 --cpu-reverse-poses 0 > gpurun_out/rev/r$K.json 2> gpurun_out/rev/r$K.err || { echo BENCHFAIL $K; tail gpurun_out/rev/r$K.err; exit 2; }
  python3 -c "import json; d=json.load(open('gpurun_out/rev/r$K.json'))['secondary']['reverse_ray_trace_fast']; r=d['roofline']; print('$K', 'ms %.3f'%d['ms_per_batch'], 'frac %.3f'%r['frac'], 'l2hit %.3f'%r['l2_hit_rate'], 'beyondL2 %.2f GB'%(r['hbm_bytes_per_launch']/1e9), r['kernel'])"
done
echo ALLOK
