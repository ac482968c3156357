#!/usr/bin/env python3
"""Per-kernel, per-dispatch averages of every counter in the rocprofv3 --pmc output
directories under <root> (pmc*/ or p*/): one line per dmf:: kernel and counter."""
import collections
import csv
import glob
import os
import sys

root = sys.argv[1]
tot = collections.defaultdict(float)
nd = collections.defaultdict(set)
for f in glob.glob(os.path.join(root, "p*", "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "")
        if not k.startswith("dmf::"):
            continue
        tot[(k, r["Counter_Name"])] += float(r["Counter_Value"])
        nd[(k, r["Counter_Name"])].add(r["Dispatch_Id"])
for (k, c), v in sorted(tot.items()):
    print(f"{k[:40]:40s} {c:24s} {v / max(len(nd[(k, c)]), 1):.4e}")
