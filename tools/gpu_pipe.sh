# Pipelined pose batches (DMF_BK_PIPE): brick parity tests with the call cut into 2 and 3
# batches, then a bench line per chunk count ($PIPES) and one kernel trace.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/pipe
export TMPDIR=/tmp
for C in ${TESTPIPES:-2 3}; do
  DMF_BK_PIPE=$C timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_boundary.py -m gpu -x -q --timeout 120 --timeout-method thread -k "${TESTK:-brick or multi_batch or never_blocks}" > gpurun_out/pipe/tests$C.log 2>&1 || { echo TESTFAIL $C; tail -30 gpurun_out/pipe/tests$C.log; exit 1; }
  tail -1 gpurun_out/pipe/tests$C.log
done
for C in ${PIPES:-1 2 3 4}; do
  DMF_BK_PIPE=$C timeout -k 10 200 python3 bench.py --steps ${STEPS:-100} --warmup 5 --cpu-frames 0 --no-secondary --pmc off ${BENCHARGS} > gpurun_out/pipe/p$C.json 2> gpurun_out/pipe/p$C.err || { echo BENCHFAIL $C; tail gpurun_out/pipe/p$C.err; exit 2; }
  python3 -c "import json,sys; d=json.load(open('gpurun_out/pipe/p$C.json')); print('pipe $C', '%.3e'%d['value'], 'step %.3f'%d['ms_per_step'], 'fuse %.3f'%d['roofline']['kernel_ms'], '%.3f'%d['roofline']['frac'])"
done
if [ -n "$TRACE" ]; then
  DMF_BK_PIPE=$TRACE timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pipe/trace -o run -- python3 bench.py --steps 5 --warmup 2 --cpu-frames 0 --no-secondary --pmc off ${BENCHARGS} > gpurun_out/pipe/trace.json 2> gpurun_out/pipe/trace.err || { echo TRACEFAIL; exit 3; }
  grep -h -E "k_bk" gpurun_out/pipe/trace/*kernel_stats.csv | awk -F'","' '{printf "%s calls=%s avg_ms=%.3f\n", substr($1,1,40), $3, $4/1e6}'
fi
echo ALLOK
