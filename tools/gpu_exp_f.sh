# Phase-F walk experiments (build_exp libraries named in F_LIBS) against the product,
# alternating on one box: 512^3 x 128 frames serial + pipelined, config 2 pipelined; digests
# show whether each stays exact.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/exp_f
mkdir -p $OUT
for name in product ${F_LIBS:-d3 d3u8 u8} product ${F_LIBS:-d3 d3u8 u8} product; do
  if [ "$name" = product ]; then lib=depth-map-fusion-utils_amd/build/libdmf.so; else lib=depth-map-fusion-utils_amd/build_exp/$name/libdmf.so; fi
  i=$((i+1))
  DMF_LIB=$lib timeout -k 10 200 python3 tools/exp_fuse.py --tag $name --calls 30 > $OUT/${name}_$i.json 2> $OUT/${name}_$i.err || { echo "FAIL $name"; tail -5 $OUT/${name}_$i.err; exit 2; }
  DMF_LIB=$lib timeout -k 10 200 python3 tools/exp_fuse.py --tag cfg2_$name --grid 256 --poses 64 --calls 60 --modes pipelined > $OUT/cfg2_${name}_$i.json 2> $OUT/cfg2_${name}_$i.err || { echo "FAIL cfg2 $name"; exit 3; }
  python3 - $OUT/${name}_$i.json $OUT/cfg2_${name}_$i.json <<'PY'
import json, sys
a, b = (json.load(open(f)) for f in sys.argv[1:3])
print(f"{a['tag']:10s} serial {a['serial_ms']:.3f} pipelined {a['pipelined_ms']:.3f} exact {a['serial_digest'] == a['pipelined_digest'] == '36708f70245952ff'}  cfg2 {b['pipelined_ms']:.3f} exact {b['digest'] == '605646542483b87f'}")
PY
done
echo FOK
