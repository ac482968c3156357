# Config 2 (256^3, 64 frames) knob sweep, pipelined, alternating with the defaults.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/exp_cfg2
mkdir -p $OUT
for rep in 1 2; do
  for k in none ${KNOBS:-span=16 span=24}; do
    kk=""; [ "$k" != none ] && kk="--knob $k"
    timeout -k 10 200 python3 tools/exp_fuse.py --tag "cfg2_$k" --grid 256 --poses 64 --calls 100 --modes pipelined $kk > $OUT/${k}_$rep.json 2> $OUT/${k}_$rep.err || { echo "FAIL $k"; exit 3; }
    python3 -c "import json; b=json.load(open('$OUT/${k}_$rep.json')); print('$k', round(b['pipelined_ms'],4), b['digest']=='605646542483b87f')"
  done
done
echo CFG2OK
