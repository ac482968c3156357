# Pass-B diagnostics: the product library and diagnostic builds (wrong results by design
# except F64) timed serially and pipelined, each under rocprofv3 --kernel-trace for the
# per-kernel averages.  Libraries are prebuilt in depth-map-fusion-utils_amd/build_exp/<name>.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/exp_b
mkdir -p $OUT
for name in product ${EXP_LIBS}; do
  if [ "$name" = product ]; then lib=depth-map-fusion-utils_amd/build/libdmf.so; else lib=depth-map-fusion-utils_amd/build_exp/$name/libdmf.so; fi
  DMF_LIB=$lib timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt_$name -o run -- python3 tools/exp_fuse.py --tag $name ${EXP_ARGS} > $OUT/$name.json 2> $OUT/$name.err || { echo "FAIL $name"; tail -5 $OUT/$name.err; exit 1; }
  cat $OUT/$name.json
  python3 tools/kt_summary.py $OUT/kt_$name 2>/dev/null | head -12
done
echo EXPOK
