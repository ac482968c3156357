# Forward march lattice mapping: 8x8 pixel tiles per wave (product) vs rows of 64 pixels
# (build_exp/rows): parity of the forward family, then the bench's secondary forward line.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/exp_fwd
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "forward or ray_trace or rayTrace" tests/test_reference_driver.py tests/test_gpu_compat.py > $O/tests.txt 2>&1 || { echo TESTFAIL; tail -20 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
for name in rows product rows product; do
  i=$((i+1))
  if [ "$name" = product ]; then lib=depth-map-fusion-utils_amd/build/libdmf.so; else lib=depth-map-fusion-utils_amd/build_exp/$name/libdmf.so; fi
  DMF_LIB=$lib timeout -k 10 300 python3 bench.py --steps 20 --warmup 2 --pmc off --cpu-frames 0 --cpu-reverse-poses 0 --serial-ref off > $O/${name}_$i.json 2> $O/${name}_$i.err || { echo "FAIL $name"; tail -5 $O/${name}_$i.err; exit 2; }
  python3 -c "import json; b=json.load(open('$O/${name}_$i.json')); s=b['secondary']; f=s['forward_first_hits']; print('$name', {k: f[k] for k in f if 'ms' in k}, s['reverse_ray_trace_fast']['ms_per_batch'])"
done
echo FWDOK
