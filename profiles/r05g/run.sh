#!/bin/bash
# Round 5: cost of pass B's store guard: product (slot clamped onto a spare record) vs no
# guard (guard0) vs a branch around the stores (guard1), 512^3 x 128 frames, alternating;
# per-kernel B time from a kernel trace of each; the guard test on the product.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r05g
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_pipeline.py -m gpu -x -v --timeout 240 --timeout-method thread -k "layout_guard" > $O/tests.log 2>&1 || { echo TESTFAIL; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
B=depth-map-fusion-utils_amd
for rep in 1 2; do
  for lib in product guard0 guard1; do
    L=$B/build/libdmf.so; [ $lib != product ] && L=$B/build_exp/$lib/libdmf.so
    DMF_LIB=$L timeout -k 10 200 python3 tools/exp_fuse.py --tag $lib --calls 40 > $O/${lib}_$rep.json 2> $O/${lib}_$rep.err || { echo "FAIL $lib"; tail -5 $O/${lib}_$rep.err; exit 3; }
    python3 -c "import json; b=json.load(open('$O/${lib}_$rep.json')); print('$lib', round(b['serial_ms'],4), round(b['pipelined_ms'],4), b['digest']=='36708f70245952ff')"
  done
done
for lib in product guard0 guard1; do
  L=$B/build/libdmf.so; [ $lib != product ] && L=$B/build_exp/$lib/libdmf.so
  DMF_LIB=$L timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_$lib -o run -- python3 tools/exp_fuse.py --calls 20 --modes serial > /dev/null 2> $O/kt_$lib.err || { echo KTFAIL; exit 4; }
  python3 -c "
import csv,glob
f=glob.glob('$O/kt_$lib/**/*kernel_stats.csv', recursive=True)[0]
for r in csv.DictReader(open(f)):
    if 'bk_pairs' in r['Name'] or 'bk_fuse_s' in r['Name'] or 'bk_rays' in r['Name']: print('$lib', r['Name'][:30], round(float(r['AverageNs'])/1e6,4))
"
done
echo ALLOK
