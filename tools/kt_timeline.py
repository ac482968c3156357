"""Timeline of a pipelined fusion run from a rocprofv3 --kernel-trace directory
(DESIGN.md §5.10): per phase-F launch, how long F ran alone, how long the next call's
A / B ran beside it, and how long A / B / the small kernels ran with no F at all.

usage: python tools/kt_timeline.py <rocprof dir> [skip_first_calls]"""
import csv
import glob
import os
import sys


def load(d):
    files = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
    if not files:
        sys.exit("no kernel_trace.csv under " + d)
    rows = []
    for r in csv.DictReader(open(files[0])):
        name = r["Kernel_Name"]
        if "dmf::" not in name:
            continue
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name.split("(")[0].replace("void ", "")))
    rows.sort()
    return rows


def union(iv):
    iv = sorted(iv)
    out = []
    for a, b in iv:
        if out and a <= out[-1][1]:
            out[-1][1] = max(out[-1][1], b)
        else:
            out.append([a, b])
    return out


def measure(iv):
    return sum(b - a for a, b in iv)


def inter(u, v):
    i = j = 0
    out = []
    while i < len(u) and j < len(v):
        a, b = max(u[i][0], v[j][0]), min(u[i][1], v[j][1])
        if a < b:
            out.append([a, b])
        if u[i][1] < v[j][1]:
            i += 1
        else:
            j += 1
    return out


def main():
    d = sys.argv[1]
    skip = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    rows = load(d)
    fs = [r for r in rows if "k_bk_fuse" in r[2]]
    if len(fs) <= skip + 2:
        sys.exit("too few phase-F launches")
    t0, t1 = fs[skip][0], fs[-2][1]  # steady window: from a phase F start to a later F end
    win = [r for r in rows if r[0] >= t0 and r[1] <= t1]
    nF = sum(1 for r in win if "k_bk_fuse" in r[2])
    kinds = {"F": lambda n: "k_bk_fuse" in n, "B": lambda n: "k_bk_pairs" in n, "A": lambda n: "k_bk_rays" in n,
             "fin/clear": lambda n: "k_finalize" in n or "fill" in n.lower() or "zero" in n.lower(),
             "small": lambda n: any(k in n for k in ("k_bk_scan", "k_bk_batch", "k_pose_table", "k_stats"))}
    U = {k: union([[a, b] for a, b, n in win if f(n)]) for k, f in kinds.items()}
    span = t1 - t0
    allu = union([[a, b] for a, b, n in win])
    print(f"window {span / 1e6:.3f} ms over {nF} phase-F launches: {span / nF / 1e6:.4f} ms per call")
    for k, u in U.items():
        print(f"  {k:10s} busy {measure(u) / nF / 1e6:.4f} ms per call")
    fo = U["F"]
    print(f"  F with B beside it   {measure(inter(fo, U['B'])) / nF / 1e6:.4f} ms per call")
    print(f"  F with A beside it   {measure(inter(fo, U['A'])) / nF / 1e6:.4f} ms per call")
    ab = union(U["A"] + U["B"])
    ab_alone = measure(ab) - measure(inter(ab, fo))
    print(f"  A or B with no F     {ab_alone / nF / 1e6:.4f} ms per call")
    print(f"  no fusion kernel     {(span - measure(allu)) / nF / 1e6:.4f} ms per call")
    per = {}
    for a, b, n in win:
        per.setdefault(n, []).append(b - a)
    for n, v in sorted(per.items(), key=lambda kv: -sum(kv[1])):
        print(f"  {n[:64]:64s} x{len(v):4d} avg {sum(v) / len(v) / 1e6:.4f} ms")


if __name__ == "__main__":
    main()
