# Pass B replaying pass A's recorded crossing paths (product) vs the previous build (prev:
# pass B re-walks): fusion parity tests, then pipelined calls under a kernel trace and
# config 2, alternating the two libraries on one box.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/exp_path
mkdir -p $OUT
timeout -k 10 500 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "fuse" tests/test_gpu_pipeline.py tests/test_gpu_configs.py > $OUT/tests.txt 2>&1 || { echo TESTFAIL; tail -30 $OUT/tests.txt; exit 1; }
tail -2 $OUT/tests.txt
for name in prev product prev product; do
  if [ "$name" = product ]; then lib=depth-map-fusion-utils_amd/build/libdmf.so; else lib=depth-map-fusion-utils_amd/build_exp/$name/libdmf.so; fi
  i=$((i+1))
  DMF_LIB=$lib timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt_${name}_$i -o run -- python3 tools/exp_fuse.py --tag $name --calls 30 > $OUT/${name}_$i.json 2> $OUT/${name}_$i.err || { echo "FAIL $name"; tail -5 $OUT/${name}_$i.err; exit 2; }
  cat $OUT/${name}_$i.json
  python3 tools/kt_summary.py $OUT/kt_${name}_$i | head -4
  DMF_LIB=$lib timeout -k 10 200 python3 tools/exp_fuse.py --tag cfg2_$name --grid 256 --poses 64 --calls 60 --modes pipelined > $OUT/cfg2_${name}_$i.json 2> $OUT/cfg2_${name}_$i.err || { echo "FAIL cfg2 $name"; exit 3; }
  cat $OUT/cfg2_${name}_$i.json
done
echo PATHOK
