# Fusion bench line + kernel trace per experiment library ($EXPS: build_exp/<name>; "base" = build/)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/exp
for E in ${EXPS:-base}; do
  if [ "$E" = base ]; then LIB=depth-map-fusion-utils_amd/build/libdmf.so; else LIB=depth-map-fusion-utils_amd/build_exp/$E/libdmf.so; fi
  DMF_LIB=$LIB timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/exp/$E -o run -- python3 bench.py --steps 5 --warmup 2 --cpu-frames 0 --no-secondary ${BENCHARGS} > gpurun_out/exp/$E.json 2> gpurun_out/exp/$E.err || { echo BENCHFAIL $E; tail gpurun_out/exp/$E.err; exit 2; }
  python3 - "$E" <<'PY'
import csv, sys
e = sys.argv[1]
for r in csv.DictReader(open(f"gpurun_out/exp/{e}/run_kernel_stats.csv")):
    if "k_bk" in r["Name"] or "k_fuse" in r["Name"]:
        print(e, r["Name"].split("(")[0].replace("void ", "")[:48], "%.3f" % (float(r["AverageNs"]) / 1e6))
PY
done
echo ALLOK
