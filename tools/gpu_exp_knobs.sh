# Runtime-knob sweep (dmf_diag.h knobs, product library), alternating with the defaults on
# one box: pipelined calls at 512^3 x 128 frames and at config 2 (256^3 x 64).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/exp_knobs
mkdir -p $OUT
for rep in 1 2; do
  for k in none ${KNOBS:-span=32 span=48 span=96 span=128}; do
    kk=""; [ "$k" != none ] && kk="--knob $k"
    timeout -k 10 200 python3 tools/exp_fuse.py --tag "$k" --calls 40 --modes pipelined $kk > $OUT/${k}_$rep.json 2> $OUT/${k}_$rep.err || { echo "FAIL $k"; tail -5 $OUT/${k}_$rep.err; exit 2; }
    timeout -k 10 200 python3 tools/exp_fuse.py --tag "cfg2_$k" --grid 256 --poses 64 --calls 60 --modes pipelined $kk > $OUT/cfg2_${k}_$rep.json 2> $OUT/cfg2_${k}_$rep.err || { echo "FAIL cfg2 $k"; exit 3; }
    python3 - $OUT/${k}_$rep.json $OUT/cfg2_${k}_$rep.json <<'PY'
import json, sys
a, b = (json.load(open(f)) for f in sys.argv[1:3])
print(f"{a['tag']:16s} pipelined {a['pipelined_ms']:.3f} exact {a['digest'] == '36708f70245952ff'}  cfg2 {b['pipelined_ms']:.3f} exact {b['digest'] == '605646542483b87f'}")
PY
  done
done
echo KNOBSOK
