#!/usr/bin/env python3
"""Per-kernel, per-dispatch PMC table of a tools/gpu_pmc_var.sh output directory."""
import collections
import csv
import glob
import os
import sys

root = sys.argv[1]
for vd in sorted(glob.glob(os.path.join(root, "v*"))):
    tot = collections.defaultdict(float)
    nd = collections.defaultdict(set)
    for f in glob.glob(os.path.join(vd, "p*", "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0].replace("void ", "")
            if "k_bk" not in k and "k_fuse" not in k:
                continue
            tot[(k, r["Counter_Name"])] += float(r["Counter_Value"])
            nd[(k, r["Counter_Name"])].add(r["Dispatch_Id"])
    print(os.path.basename(vd))
    for (k, c), v in sorted(tot.items()):
        print(f"  {k[:34]:34s} {c:24s} {v / max(len(nd[(k, c)]), 1):.4e}")
