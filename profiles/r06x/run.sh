#!/bin/bash
# Round 6: the refill's adoption adds issued after its record fetch (late, DMF_EXP_F_LATE_ADOPT)
# alternating, headline and config 2, then kernel traces
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r06x
mkdir -p $O
B=depth-map-fusion-utils_amd
LIBS="product late"
for rep in 1 2 3; do
  for lib in $LIBS; do
    L=$B/build/libdmf.so; [ $lib != product ] && L=$B/build_exp/$lib/libdmf.so
    DMF_LIB=$L timeout -k 10 200 python3 tools/exp_fuse.py --tag $lib --calls 60 > $O/c4_${lib}_$rep.json 2> $O/c4_${lib}_$rep.err || { echo "FAIL $lib"; tail -5 $O/c4_${lib}_$rep.err; exit 3; }
    DMF_LIB=$L timeout -k 10 200 python3 tools/exp_fuse.py --tag $lib --grid 256 --poses 64 --calls 150 > $O/c2_${lib}_$rep.json 2> /dev/null || { echo "FAIL $lib"; exit 3; }
    python3 -c "import json; b=json.load(open('$O/c4_${lib}_$rep.json')); c=json.load(open('$O/c2_${lib}_$rep.json')); print('$lib', round(b['serial_ms'],4), round(b['pipelined_ms'],4), b['digest']=='36708f70245952ff', round(c['serial_ms'],4), round(c['pipelined_ms'],4), c['digest']=='605646542483b87f')"
  done
done
for lib in $LIBS; do
  L=$B/build/libdmf.so; [ $lib != product ] && L=$B/build_exp/$lib/libdmf.so
  DMF_LIB=$L timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_$lib -o run -- python3 tools/exp_fuse.py --calls 20 --modes serial > /dev/null 2> $O/kt_$lib.err || { echo "KTFAIL $lib"; exit 4; }
  python3 -c "
import csv; r=list(csv.DictReader(open('$O/kt_$lib/run_kernel_stats.csv')))
print('$lib', {x['Name'].split('(')[0].replace('void ','')[-28:]:round(float(x['AverageNs'])/1e6,4) for x in r if 'k_bk_' in x['Name'] and ('pairs' in x['Name'] or 'fuse_s' in x['Name'] or 'rays' in x['Name'])})"
done
echo ALLOK
