#!/bin/bash
# Round 5: forward first hits per-XCD queues (fwd_kernel 1) vs the grid (0): parity, A/B, PMC.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r05c
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 200 --timeout-method thread -k "batched_device or reverse_fast_parity" > $O/parity.log 2>&1 || { echo PARITYFAIL; tail -30 $O/parity.log; exit 1; }
tail -2 $O/parity.log
timeout -k 10 300 python tools/exp_forward.py 0,1,0,1,0,1 > $O/ab.json 2> $O/ab.err || { echo ABFAIL; tail -20 $O/ab.err; exit 2; }
cat $O/ab.json
for k in 0 1; do
  for pass in "SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES TCC_HIT_sum TCC_MISS_sum" "FETCH_SIZE" "WRITE_SIZE"; do
    tag=$(echo $pass | cut -c1-8)
    timeout -k 10 180 rocprofv3 --pmc $pass --output-format csv -d $O/pmc_k${k}_$tag -o run -- python tools/exp_forward.py $k > /dev/null 2> $O/pmc_k${k}_$tag.err || { echo PMCFAIL $k $tag; tail -5 $O/pmc_k${k}_$tag.err; exit 3; }
  done
done
echo ALLOK
