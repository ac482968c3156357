# Phase F with every LDS add unmasked (experiment builds): a cell the lane does not own goes
# to an address past the workgroup's LDS (f_oob1) or to a per-lane dummy word (f_oob2), so
# the slab walk has no exec-mask changes.  Digests show whether the results stay exact.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/exp_oob
mkdir -p $OUT
for name in product f_oob1 f_oob2 product f_oob1 f_oob2; do
  if [ "$name" = product ]; then lib=depth-map-fusion-utils_amd/build/libdmf.so; else lib=depth-map-fusion-utils_amd/build_exp/$name/libdmf.so; fi
  i=$((i+1))
  DMF_LIB=$lib timeout -k 10 200 python3 tools/exp_fuse.py --tag $name --calls 30 > $OUT/${name}_$i.json 2> $OUT/${name}_$i.err || { echo "FAIL $name"; tail -5 $OUT/${name}_$i.err; exit 2; }
  cat $OUT/${name}_$i.json
  DMF_LIB=$lib timeout -k 10 200 python3 tools/exp_fuse.py --tag cfg2_$name --grid 256 --poses 64 --calls 60 --modes pipelined > $OUT/cfg2_${name}_$i.json 2> $OUT/cfg2_${name}_$i.err || { echo "FAIL cfg2 $name"; exit 3; }
  cat $OUT/cfg2_${name}_$i.json
done
echo OOBOK
