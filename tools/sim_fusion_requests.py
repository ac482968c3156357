#!/usr/bin/env python3
"""CPU model of the fusion kernel's memory-side atomic requests.

Rays of random PX x PY pixel packets (rendered scene, 512^3 grid) are walked with the
exact DDA of oracle/py_oracle.py in rounds of S updates; per round it reports
  updates per distinct cell  (LDS aggregation factor),
  distinct cells per 64-B counter line for several counter layouts,
  requests per update, and the distribution of the round's box volume.
usage: tools/sim_fusion_requests.py PX PY S[,S...]     (e.g. 8 8 10,14)
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "depth-map-fusion-utils_amd")]
import numpy as np  # noqa: E402

from dmf_amd import scene  # noqa: E402
from oracle import py_oracle as PY  # noqa: E402

LAYOUTS = {
    "x-major rows (16 z)": lambda c: (c[0], c[1], c[2] // 16),
    "tile 1x4x4": lambda c: (c[0], c[1] // 4, c[2] // 4),
    "tile 2x2x4": lambda c: (c[0] // 2, c[1] // 2, c[2] // 4),
}


def main():
    PX, PYk = int(sys.argv[1]), int(sys.argv[2])
    Ss = [int(x) for x in sys.argv[3].split(",")]
    K = scene.K_640x480
    W, H = 640, 480
    poses = scene.fibonacci_poses(4, seed=1234)
    depth = scene.render_frames(K, W, H, poses)
    v = PY.Vol((-0.5, 0.5, -0.5, 0.5, -0.5, 0.5), (512, 512, 512))
    rng = np.random.default_rng(0)
    res = {S: {"vol": [], "upd": 0, "cells": 0, "lines": {k: 0 for k in LAYOUTS}} for S in Ss}
    npk = 0
    while npk < 40:
        p = int(rng.integers(0, 4))
        r0, c0 = int(rng.integers(0, H // PYk)) * PYk, int(rng.integers(0, W // PX)) * PX
        T = poses[p]
        O = (np.float32(T[3]), np.float32(T[7]), np.float32(T[11]))
        rays = []
        for r in range(r0, r0 + PYk):
            for c in range(c0, c0 + PX):
                d = int(depth[p, r, c])
                if not (scene.DEPTH_MIN_MM <= d < scene.DEPTH_MAX_MM):
                    continue
                E = PY.transform(T, PY.project_point(K, r, c, d))
                inside = v.valid_points(E) and v.valid_coords(v.get_voxel(E))
                rays.append(PY.dda_cells(v, O, E, inside)[0])
        if len(rays) < PX * PYk // 2:
            continue
        npk += 1
        L = max(len(m) for m in rays)
        for S in Ss:
            R = res[S]
            for k0 in range(0, L, S):
                cells = set()
                for m in rays:
                    seg = m[k0:k0 + S]
                    R["upd"] += len(seg)
                    cells.update(seg)
                if not cells:
                    continue
                a = np.array(list(cells))
                R["vol"].append(int(np.prod(a.max(0) - a.min(0) + 1)))
                R["cells"] += len(cells)
                for k, f in LAYOUTS.items():
                    R["lines"][k] += len({f(cc) for cc in cells})
    for S in Ss:
        R = res[S]
        vv = np.array(R["vol"])
        print(f"packet {PX}x{PYk} S={S}: updates/cell {R['upd'] / R['cells']:.2f}  box vol p50 "
              f"{np.percentile(vv, 50):.0f} p99 {np.percentile(vv, 99):.0f} max {vv.max()}")
        for k in LAYOUTS:
            print(f"   {k:22s} cells/line {R['cells'] / R['lines'][k]:.2f}  requests/update "
                  f"{R['lines'][k] / R['upd']:.4f}")


if __name__ == "__main__":
    main()
