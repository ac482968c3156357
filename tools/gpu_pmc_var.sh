# PMC passes (one counter group per run) of the fusion pipeline per fusion variant ($VARIANTS)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/pmcv
for V in ${VARIANTS:-0}; do
  i=0; mkdir -p gpurun_out/pmcv/v$V
  for pmc in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU" "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INST_CYCLES_SALU" ${EXTRA_PMC}; do
    i=$((i+1))
    DMF_FUSE_VARIANT=$V timeout -k 10 120 rocprofv3 --pmc $pmc --output-format csv -d gpurun_out/pmcv/v$V/p$i -o run -- python3 bench.py --steps 1 --warmup 0 --cpu-frames 0 --no-secondary ${BENCHARGS} > gpurun_out/pmcv/v$V/p$i.json 2> gpurun_out/pmcv/v$V/p$i.err || { echo PMCFAIL $V $i; tail -5 gpurun_out/pmcv/v$V/p$i.err; exit 1; }
  done
done
python3 tools/pmc_table.py gpurun_out/pmcv
echo ALLOK
