#!/bin/bash
# Round 6: what bounds phase F -- diagnostic builds that add work to the walk: xvalu (+7
# independent VALU per slab) and xlds (every walk atomic issued twice; wrong counts) vs the
# product, alternating; kernel trace per build.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r06m
mkdir -p $O
B=depth-map-fusion-utils_amd
LIBS="product xvalu xlds"
for rep in 1 2; do
  for lib in $LIBS; do
    L=$B/build/libdmf.so; [ $lib != product ] && L=$B/build_exp/$lib/libdmf.so
    DMF_LIB=$L timeout -k 10 200 python3 tools/exp_fuse.py --tag $lib --calls 60 > $O/c4_${lib}_$rep.json 2> $O/c4_${lib}_$rep.err || { echo "FAIL $lib"; tail -5 $O/c4_${lib}_$rep.err; exit 3; }
    python3 -c "import json; b=json.load(open('$O/c4_${lib}_$rep.json')); print('$lib', round(b['serial_ms'],4), round(b['pipelined_ms'],4), b['digest']=='36708f70245952ff')"
  done
done
for lib in $LIBS; do
  L=$B/build/libdmf.so; [ $lib != product ] && L=$B/build_exp/$lib/libdmf.so
  DMF_LIB=$L timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_$lib -o run -- python3 tools/exp_fuse.py --calls 20 --modes serial > /dev/null 2> $O/kt_$lib.err || { echo "KTFAIL $lib"; exit 4; }
  python3 -c "
import csv; r=list(csv.DictReader(open('$O/kt_$lib/run_kernel_stats.csv')))
print('$lib', {x['Name'].split('(')[0].replace('void ','')[-28:]:round(float(x['AverageNs'])/1e6,4) for x in r if 'k_bk_' in x['Name'] and ('pairs' in x['Name'] or 'fuse_s' in x['Name'] or 'rays' in x['Name'])})"
done
for lib in xvalu xlds; do
  L=$B/build_exp/$lib/libdmf.so
  DMF_LIB=$L timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT --output-format csv -d $O/pmc_$lib -o run -- python3 tools/exp_fuse.py --calls 3 --modes serial > /dev/null 2> $O/pmc_$lib.err || { echo PMCFAIL; exit 5; }
  python3 - $O/pmc_$lib <<'PY'
import csv, glob, collections, sys
t = collections.defaultdict(float); n = set()
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "k_bk_fuse_s" in r["Kernel_Name"]:
            t[r["Counter_Name"]] += float(r["Counter_Value"]); n.add(r["Dispatch_Id"])
print(sys.argv[1], {x: round(v / len(n) / 1e9, 4) for x, v in sorted(t.items())})
PY
done
echo ALLOK
