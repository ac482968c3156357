# A/B: bench (no secondary, no CPU) with each experiment library, plus a kernel trace per library
set -o pipefail
mkdir -p gpurun_out/exp
export TMPDIR=/tmp
for E in base ${EXPS}; do
  if [ "$E" = base ]; then LIB=depth-map-fusion-utils_amd/build/libdmf.so; else LIB=depth-map-fusion-utils_amd/build_exp/$E/libdmf.so; fi
  DMF_LIB=$LIB timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/exp/$E -o run -- python3 bench.py --steps 3 --warmup 1 --cpu-frames 0 --no-secondary > gpurun_out/exp/$E.json 2> gpurun_out/exp/$E.err || { echo EXPFAIL $E; exit 1; }
done
echo ALLOK
