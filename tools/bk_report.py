"""Summarise tools/gpu_bk_iter.sh output: bench lines per variant and PMC per brick kernel."""
import csv, collections, glob, json, sys
for f in sorted(glob.glob("gpurun_out/bk_bench_*.json")):
    d = json.load(open(f))
    print(f.split("_")[-1][:-5], f"{d['value']/1e9:.1f} Gupd/s", {k: round(v, 3) for k, v in d["step_breakdown_ms"].items()})
tot = collections.defaultdict(float)
for r in csv.DictReader(open("gpurun_out/bk_pmc/it/run_counter_collection.csv")):
    k = r["Kernel_Name"].split("(")[0].replace("void ", "")
    if k.startswith("dmf::"):
        tot[(k, r["Counter_Name"])] += float(r["Counter_Value"])
for (k, c), v in sorted(tot.items()):
    print(f"{k:28s} {c:24s} {v:.4g}")
