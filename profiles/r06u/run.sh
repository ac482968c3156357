#!/bin/bash
# Round 6: what paces pass B -- a diagnostic build without its per-pair slot atomics (noslot:
# plain LDS reads, the layout check then fails and phase F skips the batch; wrong results) vs
# the product, pass B's kernel time in a serial-call trace, and pass B's counters.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r06u
mkdir -p $O
B=depth-map-fusion-utils_amd
for lib in product noslot product noslot; do
  L=$B/build/libdmf.so; [ $lib != product ] && L=$B/build_exp/$lib/libdmf.so
  i=$((i+1))
  DMF_LIB=$L timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_${lib}_$i -o run -- python3 tools/exp_fuse.py --calls 20 --modes serial > /dev/null 2> $O/kt_${lib}_$i.err || { echo "KTFAIL $lib"; exit 4; }
  python3 -c "
import csv; r=list(csv.DictReader(open('$O/kt_${lib}_$i/run_kernel_stats.csv')))
print('$lib', {x['Name'].split('(')[0].replace('void ','')[-28:]:round(float(x['AverageNs'])/1e6,4) for x in r if 'k_bk_' in x['Name'] and ('pairs' in x['Name'] or 'fuse_s' in x['Name'] or 'rays' in x['Name'])})"
done
for lib in product noslot; do
  L=$B/build/libdmf.so; [ $lib != product ] && L=$B/build_exp/$lib/libdmf.so
  DMF_LIB=$L timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT --output-format csv -d $O/pmc_$lib -o run -- python3 tools/exp_fuse.py --calls 3 --modes serial > /dev/null 2> $O/pmc_$lib.err || { echo PMCFAIL; exit 5; }
  python3 - $O/pmc_$lib <<'PY'
import csv, glob, collections, sys
t = collections.defaultdict(float); n = set()
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "k_bk_pairs" in r["Kernel_Name"]:
            t[r["Counter_Name"]] += float(r["Counter_Value"]); n.add(r["Dispatch_Id"])
print(sys.argv[1], {x: round(v / len(n) / 1e9, 4) for x, v in sorted(t.items())})
PY
done
echo ALLOK
