#!/bin/bash
# Round 6: where the pipelined step goes after the slab code and the atomic-optimizer change:
# kernel-trace timeline of pipelined calls, phase F's in-kernel phase timers (DMF_EXP_STATS
# build), phase F's PMC (issue / wait / LDS), and the trace kernels without the atomic
# optimizer (tnao) vs the product.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r06c
mkdir -p $O
B=depth-map-fusion-utils_amd
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/kt_pipe -o run -- python3 tools/exp_fuse.py --calls 40 --modes pipelined > $O/kt_pipe.json 2> $O/kt_pipe.err || { echo KTFAIL; tail -5 $O/kt_pipe.err; exit 1; }
python3 tools/kt_timeline.py $O/kt_pipe 10 > $O/timeline.txt 2>&1; tail -15 $O/timeline.txt
DMF_LIB=$B/build_exp/stats/libdmf.so timeout -k 10 300 python3 bench.py --steps 100 --no-secondary --cpu-frames 0 --pmc off --serial-ref off > $O/bench_stats.json 2> $O/bench_stats.err || { echo STATSFAIL; tail -5 $O/bench_stats.err; exit 2; }
python3 -c "import json; b=json.load(open('$O/bench_stats.json')); print(json.dumps(b['fuse_diagnostics']))"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT --output-format csv -d $O/pmc_f -o run -- python3 tools/exp_fuse.py --calls 3 --modes serial > /dev/null 2> $O/pmc_f.err || { echo PMCFAIL; tail -5 $O/pmc_f.err; exit 3; }
python3 - <<'PY'
import csv, glob, collections
t = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.defaultdict(set)
for f in glob.glob("gpurun_out/r06c/pmc_f/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "")
        if "k_bk_" in k:
            t[k][r["Counter_Name"]] += float(r["Counter_Value"]); n[k].add(r["Dispatch_Id"])
for k, c in t.items():
    d = len(n[k]); print(k, d, {x: round(v / d / 1e9, 4) for x, v in sorted(c.items())})
PY
for rep in 1 2; do
  for lib in product tnao; do
    L=$B/build/libdmf.so; [ $lib != product ] && L=$B/build_exp/$lib/libdmf.so
    DMF_LIB=$L timeout -k 10 200 python3 tools/exp_reverse.py 0 > $O/rev_${lib}_$rep.json 2> /dev/null || { echo "REVFAIL $lib"; exit 4; }
    DMF_LIB=$L timeout -k 10 200 python3 tools/exp_forward.py 0 > $O/fwd_${lib}_$rep.json 2> /dev/null || { echo "FWDFAIL $lib"; exit 4; }
    echo "$lib $(cat $O/rev_${lib}_$rep.json | head -c 400)"; echo "$lib $(cat $O/fwd_${lib}_$rep.json | head -c 300)"
  done
done
echo ALLOK
