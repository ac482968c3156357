#!/usr/bin/env python3
"""Summarise a tools/profile_round.sh output directory into profiles/<tag>/.

Writes kernel_stats.csv (rocprofv3 --stats), pmc_per_kernel.csv (counter totals per
kernel, per dispatch) and, for the fusion kernel, profiles/pmc_fuse_summary.json with
HBM bytes per launch:  traffic = (2 * FETCH_SIZE + WRITE_SIZE) * 1024.
FETCH_SIZE is doubled per MI355X_MICROARCH.md §HBM (gfx950 tallies 128-B requests at
64 B); WRITE_SIZE also counts the memory-side atomics (32 B per request observed).
"""
import collections
import csv
import glob
import json
import os
import shutil
import sys

src, dst = sys.argv[1], sys.argv[2]
os.makedirs(dst, exist_ok=True)
shutil.copy(os.path.join(src, "kt", "run_kernel_stats.csv"), os.path.join(dst, "kernel_stats.csv"))
tot = collections.defaultdict(float)
ndisp = collections.defaultdict(set)
for f in sorted(glob.glob(os.path.join(src, "pmc*", "run_counter_collection.csv")) + glob.glob(os.path.join(src, "p[0-9]*", "run_counter_collection.csv"))):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "")
        if not k.startswith("dmf::"):
            continue
        tot[(k, r["Counter_Name"])] += float(r["Counter_Value"])
        ndisp[(k, r["Counter_Name"])].add(r["Dispatch_Id"])
with open(os.path.join(dst, "pmc_per_kernel.csv"), "w", newline="") as f:
    w = csv.writer(f)  # quoted: template arguments hold commas
    w.writerow(["kernel", "counter", "total", "dispatches", "per_dispatch"])
    for (k, c), v in sorted(tot.items()):
        n = len(ndisp[(k, c)])
        w.writerow([k, c, f"{v:.0f}", n, f"{v / n:.1f}"])
if not os.path.exists(os.path.join(src, "bench_kt.json")):
    # a bench.py --pmc-dir directory (the bench line carries its own summary): counters and
    # kernel statistics only
    sys.exit(0)
bench = json.load(open(os.path.join(src, "bench_kt.json")))
# the fusion launch = every kernel of the fusion pipeline (brick path: k_bk_rays, k_bk_scan,
# k_bk_pairs, k_bk_fuse; LDS-box path: k_fuse_l alone), priced per bench step
PIPE = ("dmf::k_bk_", "dmf::k_fuse")
kernels = sorted({k for (k, c) in tot if k.startswith(PIPE)})
if kernels:
    # per fusion call (a call of a multi-batch config launches each kernel once per batch);
    # the PMC passes run their own (shorter) bench command: count its calls, not the trace's
    pmc_bench = json.load(open(sorted(glob.glob(os.path.join(src, "pmc*.json")))[0]))
    calls = int(pmc_bench["steps"]) + int(pmc_bench["warmup"])
    # a pipelined bench also re-times the serial call after its timed region (roofline.
    # serial_call_ms): count the phase-F dispatches instead (one per call and batch)
    fk = [k for k in kernels if k.startswith(("dmf::k_bk_fuse", "dmf::k_fuse"))]
    if fk and (pmc_bench.get("roofline") or {}).get("serial_call_ms"):
        calls = max(len(ndisp[(fk[0], c)]) for (k, c) in tot if k == fk[0])

    def per(k, c):
        return tot.get((k, c), 0.0) / max(calls, 1)
    per_kernel = {k: {"fetch_bytes_raw": per(k, "FETCH_SIZE") * 1024, "write_bytes": per(k, "WRITE_SIZE") * 1024,
                      "hbm_bytes": (2 * per(k, "FETCH_SIZE") + per(k, "WRITE_SIZE")) * 1024} for k in kernels}
    hbm = sum(v["hbm_bytes"] for v in per_kernel.values())
    summ = {"kernel": bench["roofline"]["kernel"], "pipeline": kernels, "grid": bench["config"]["grid"],
            "poses": bench["config"]["poses_per_gpu"], "image": bench["config"]["image"],
            "hbm_bytes_per_launch": hbm, "profile": dst,
            "per_kernel": per_kernel,
            "tcc_ea0_atomic_requests_per_launch": sum(per(k, "TCC_EA0_ATOMIC_sum") for k in kernels),
            "algorithmic_bytes_per_launch": bench["roofline"]["algorithmic_bytes_per_launch"],
            "kernel_ms_bench": bench["roofline"].get("step_ms", bench["roofline"].get("kernel_ms")),
            "note": "traffic = sum over the pipeline's kernels of (2*FETCH_SIZE + WRITE_SIZE)*1024 per launch; "
                    "FETCH doubled per MI355X_MICROARCH.md"}
    json.dump(summ, open(os.path.join(dst, "pmc_fuse_summary.json"), "w"), indent=1)
    print(json.dumps(summ, indent=1))
shutil.copy(os.path.join(src, "bench_kt.json"), os.path.join(dst, "bench_under_rocprof.json"))
# per-kernel average over the timed steps only (rocprofv3 --stats also averages the cold
# warmup dispatches): the last `steps` fusion calls of the traced bench command
trace = sorted(csv.DictReader(open(os.path.join(src, "kt", "run_kernel_trace.csv"))), key=lambda r: int(r["Start_Timestamp"]))
durs = collections.defaultdict(list)
for r in trace:
    durs[r["Kernel_Name"].split("(")[0].replace("void ", "")].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
steps, warm = int(bench["steps"]), int(bench["warmup"])
with open(os.path.join(dst, "kernel_timed_avg.csv"), "w") as f:
    w = csv.writer(f)
    w.writerow(["kernel", "dispatches_total", "dispatches_timed", "avg_ms_timed"])
    for k, v in sorted(durs.items()):
        if not k.startswith("dmf::"):
            continue
        per_call = len(v) // max(steps + warm, 1) if len(v) >= steps + warm else 0
        timed = v[-steps * per_call:] if per_call else v
        w.writerow([k, len(v), len(timed), f"{sum(timed) / len(timed):.4f}"])
