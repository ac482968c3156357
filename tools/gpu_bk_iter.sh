# one iteration of the brick-fusion loop: parity (brick tests), bench per variant, one PMC pass
set -o pipefail
mkdir -p gpurun_out/bk_pmc
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "brick" -x -q --timeout 120 --timeout-method thread > gpurun_out/bk_test.log 2>&1 || { echo TESTFAIL; tail -30 gpurun_out/bk_test.log; exit 1; }
for V in ${VARIANTS:-40}; do
  DMF_FUSE_VARIANT=$V timeout -k 10 200 python bench.py --steps 3 --warmup 1 --cpu-frames 0 --no-secondary > gpurun_out/bk_bench_$V.json 2> gpurun_out/bk_bench_$V.err || { echo BENCHFAIL $V; exit 2; }
done
export TMPDIR=/tmp DMF_FUSE_VARIANT=${PMCV:-40}
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --output-format csv -d gpurun_out/bk_pmc/it -o run -- python3 bench.py --steps 1 --warmup 0 --cpu-frames 0 --no-secondary > gpurun_out/bk_pmc/it.json 2> gpurun_out/bk_pmc/it.err || { echo PMCFAIL; exit 3; }
if [ -n "$KT" ]; then timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/bk_kt -o run -- python3 bench.py --steps 3 --warmup 1 --cpu-frames 0 --no-secondary > gpurun_out/bk_kt.json 2> gpurun_out/bk_kt.err || { echo KTFAIL; exit 4; }; fi
echo ALLOK
