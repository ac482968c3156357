# Pass-B diagnostics (wrong results by design): what B's time is made of.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/exp_b2
mkdir -p $OUT
for name in product b_uni b_stride b_defer b_defer_f64; do
  if [ "$name" = product ]; then lib=depth-map-fusion-utils_amd/build/libdmf.so; else lib=depth-map-fusion-utils_amd/build_exp/$name/libdmf.so; fi
  echo "== $name"
  DMF_LIB=$lib timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt_$name -o run -- python3 tools/exp_fuse.py --tag $name --calls 15 --modes serial > $OUT/$name.json 2> $OUT/$name.err || { echo "FAIL $name"; tail -5 $OUT/$name.err; exit 1; }
  cat $OUT/$name.json
  python3 tools/kt_summary.py $OUT/kt_$name | head -4
done
echo EXPOK
