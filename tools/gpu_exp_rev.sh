# reverseRayTraceFast work-queue shape sweep (exp_reverse.py per library; knob 0 = spatial
# order, 3 = insertion order, masks compared).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/exp_rev
mkdir -p $OUT
for name in product ${REV_LIBS:-r1024_8_8 r512_16_8 r512_8_16}; do
  if [ "$name" = product ]; then lib=depth-map-fusion-utils_amd/build/libdmf.so; else lib=depth-map-fusion-utils_amd/build_exp/$name/libdmf.so; fi
  echo "== $name"
  DMF_LIB=$lib timeout -k 10 200 python3 tools/exp_reverse.py > $OUT/$name.json 2> $OUT/$name.err || { echo "FAIL $name"; tail -5 $OUT/$name.err; exit 1; }
  cat $OUT/$name.json
done
echo REVOK
