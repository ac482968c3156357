# A/B on one box: (1) pass-B occupancy builds (build_exp/bw5, bw6 vs build/) on the fusion
# bench, alternating; (2) reverse-march arithmetic variants (DMF_REVERSE_KERNEL 2 = default,
# 9 = round-2 arithmetic, 10 = float bins only, 11 = fast division only) on the bench's
# secondary leg.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ab3
B="--steps 300 --warmup 3 --pmc off --cpu-frames 0 --cpu-reverse-poses 0 --no-secondary"
for i in 1 2; do
  for E in base bw5 bw6; do
    if [ "$E" = base ]; then LIB=depth-map-fusion-utils_amd/build/libdmf.so; else LIB=depth-map-fusion-utils_amd/build_exp/$E/libdmf.so; fi
    DMF_LIB=$LIB timeout -k 10 200 python3 bench.py $B > gpurun_out/ab3/$E$i.json 2> gpurun_out/ab3/$E$i.err || { echo BENCHFAIL $E; tail gpurun_out/ab3/$E$i.err; exit 2; }
    echo -n "$E: "; python3 tools/show_bench.py gpurun_out/ab3/$E$i.json
  done
done
for i in 1 2; do
  for V in 2 9 10 11; do
    DMF_REVERSE_KERNEL=$V timeout -k 10 200 python3 bench.py --steps 5 --warmup 1 --pmc off --cpu-frames 0 --cpu-reverse-poses 0 > gpurun_out/ab3/rev$V.$i.json 2> gpurun_out/ab3/rev$V.$i.err || { echo REVFAIL $V; tail gpurun_out/ab3/rev$V.$i.err; exit 3; }
    echo -n "rev$V: "; python3 tools/show_bench.py gpurun_out/ab3/rev$V.$i.json | tail -1
  done
done
echo AB3_OK
