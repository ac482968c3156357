"""Per-kernel average durations from a rocprofv3 --kernel-trace --stats output directory:
prints the stats table rows of the dmf:: kernels (calls, average and total ms)."""
import csv
import glob
import os
import sys

d = sys.argv[1]
files = glob.glob(os.path.join(d, "**", "*kernel_stats.csv"), recursive=True)
if not files:
    sys.exit("no kernel_stats.csv under " + d)
rows = list(csv.DictReader(open(files[0])))
for r in sorted(rows, key=lambda r: -float(r.get("TotalDurationNs", 0))):
    name = r["Name"].split("(")[0].replace("void ", "")
    if "dmf::" not in name:
        continue
    print("%-60s calls %6s  avg %8.3f ms  total %9.3f ms" % (name[:60], r["Calls"], float(r["AverageNs"]) / 1e6,
                                                            float(r["TotalDurationNs"]) / 1e6))
