# PMC passes over the brick fusion variant $V (one rocprofv3 run per counter group)
set -o pipefail
export TMPDIR=/tmp DMF_FUSE_VARIANT=${V:-40}
mkdir -p gpurun_out/bk_pmc
i=0
for pmc in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $pmc --output-format csv -d gpurun_out/bk_pmc/p$i -o run -- python3 bench.py --steps 1 --warmup 0 --cpu-frames 0 --no-secondary > gpurun_out/bk_pmc/p$i.json 2> gpurun_out/bk_pmc/p$i.err || { echo PMCFAIL $i; exit 1; }
done
echo ALLOK
