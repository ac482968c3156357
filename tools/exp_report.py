"""Summarise tools/gpu_exp.sh: fusion ms and per-kernel averages per experiment."""
import csv, glob, json, os
for f in sorted(glob.glob("gpurun_out/exp/*.json")):
    e = os.path.basename(f)[:-5]
    d = json.loads(open(f).read().strip().splitlines()[-1])
    ks = {}
    for r in csv.DictReader(open(f"gpurun_out/exp/{e}/run_kernel_stats.csv")):
        n = r["Name"].split("(")[0].replace("void ", "")
        if n.startswith("dmf::k_bk") or n.startswith("dmf::k_fuse"):
            ks[n] = round(float(r["AverageNs"]) / 1e6, 3)
    print(f"{e:12s} fuse {d['step_breakdown_ms']['fuse']:.3f} ms  {ks}")
