# Bench lines for a list of environment settings ($SETS: ';'-separated, each "VAR=V VAR2=W"
# or "-" for the defaults); fusion kernel time only.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/env
i=0
IFS=';' read -ra LIST <<< "${SETS:--}"
for S in "${LIST[@]}"; do
  i=$((i+1))
  E=""; [ "$S" != "-" ] && E="$S"
  env $E timeout -k 10 200 python3 bench.py --steps 100 --warmup 3 --pmc off --cpu-frames 0 --cpu-reverse-poses 0 --no-secondary ${BENCHARGS} > gpurun_out/env/s$i.json 2> gpurun_out/env/s$i.err || { echo BENCHFAIL "$S"; tail gpurun_out/env/s$i.err; exit 2; }
  python3 -c "import json; d=json.load(open('gpurun_out/env/s$i.json')); print('[$S]', '%.3f'%d['roofline']['kernel_ms'], d['fuse_diagnostics']['parts'])"
done
echo ALLOK
