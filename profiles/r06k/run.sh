#!/bin/bash
# Round 6: phase F's refill threshold and walk-block length re-swept after the cheaper refill
# (stride + adoption table): refill at >= 12 / 8 idle lanes (r12, r8), 6-slab blocks with 12
# (u6r12), 4-slab blocks with 8 (u4r8) vs the product (16, 8-slab blocks); alternating, headline
# and config 2; then the kernel trace per build, phase F's counters of the product, and its
# in-kernel lane statistics (DMF_EXP_STATS build).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r06k
mkdir -p $O
B=depth-map-fusion-utils_amd
LIBS="product r12 r8 u6r12 u4r8"
for rep in 1 2; do
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
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT --output-format csv -d $O/pmc_f -o run -- python3 tools/exp_fuse.py --calls 3 --modes serial > /dev/null 2> $O/pmc_f.err || { echo PMCFAIL; tail -5 $O/pmc_f.err; exit 5; }
python3 - <<'PY'
import csv, glob, collections
t = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.defaultdict(set)
for f in glob.glob("gpurun_out/r06k/pmc_f/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "")
        if "k_bk_" in k:
            t[k][r["Counter_Name"]] += float(r["Counter_Value"]); n[k].add(r["Dispatch_Id"])
for k, c in t.items():
    d = len(n[k]); print(k, d, {x: round(v / d / 1e9, 4) for x, v in sorted(c.items())})
PY
DMF_LIB=$B/build_exp/stats/libdmf.so timeout -k 10 300 python3 bench.py --steps 100 --no-secondary --cpu-frames 0 --pmc off --serial-ref off > $O/bench_stats.json 2> $O/bench_stats.err || { echo STATSFAIL; tail -5 $O/bench_stats.err; exit 6; }
python3 -c "import json; b=json.load(open('$O/bench_stats.json')); print(json.dumps(b['fuse_diagnostics']))"
echo ALLOK
