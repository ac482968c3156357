# Kernel traces of the experiment libraries $LIBS (build_exp/<name>, "default" = build/) on the
# default bench workload; per-kernel averages printed per library.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
for NAME in ${LIBS:-default}; do
  OUT=gpurun_out/ekt_$NAME
  mkdir -p "$OUT"
  LIB=depth-map-fusion-utils_amd/build/libdmf.so
  [ "$NAME" != default ] && LIB=depth-map-fusion-utils_amd/build_exp/$NAME/libdmf.so
  DMF_LIB=$LIB timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kt" -o run -- python3 bench.py --steps 20 --warmup 2 --cpu-frames 0 --cpu-reverse-poses 0 --pmc off --no-secondary ${BENCHARGS} > "$OUT/bench_kt.json" 2> "$OUT/bench_kt.err" || { echo KTFAIL $NAME; tail "$OUT/bench_kt.err"; exit 1; }
  echo "== $NAME"
  python3 tools/kt_summary.py "$OUT" | grep -E "k_bk|k_fuse" || exit 2
done
echo ALLOK
