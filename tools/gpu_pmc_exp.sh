# PMC passes (one counter group per run) of the fusion kernels for experiment libraries $EXPS
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/pmcx
for E in ${EXPS:-base}; do
  if [ "$E" = base ]; then LIB=depth-map-fusion-utils_amd/build/libdmf.so; else LIB=depth-map-fusion-utils_amd/build_exp/$E/libdmf.so; fi
  i=0; mkdir -p gpurun_out/pmcx/$E
  for pmc in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU" "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_SALU SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD"; do
    i=$((i+1))
    DMF_LIB=$LIB timeout -k 10 120 rocprofv3 --pmc $pmc --output-format csv -d gpurun_out/pmcx/$E/p$i -o run -- python3 bench.py --steps 1 --warmup 0 --cpu-frames 0 --no-secondary > gpurun_out/pmcx/$E/p$i.json 2> gpurun_out/pmcx/$E/p$i.err || { echo PMCFAIL $E $i; tail -5 gpurun_out/pmcx/$E/p$i.err; exit 1; }
  done
done
echo ALLOK
