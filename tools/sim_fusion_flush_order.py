#!/usr/bin/env python3
"""CPU model: memory-side atomic requests of the fusion flush by LIST ORDER.

The hardware issues one request per distinct 64-B counter line per wave instruction,
so the order of the compacted (cell, count) list matters: each 64-entry chunk costs
the number of distinct lines it touches.  Rays of random 8x8 packets (rendered
scene, 512^3 grid) are walked with the exact DDA of oracle/py_oracle.py in rounds of
S updates; for each list order x global counter layout it reports requests/update.
usage: tools/sim_fusion_flush_order.py [S] [packets]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "depth-map-fusion-utils_amd")]
import numpy as np
from dmf_amd import scene
from oracle import py_oracle as PY
K = scene.K_640x480; W, H = 640, 480
poses = scene.fibonacci_poses(4, seed=1234)
depth = scene.render_frames(K, W, H, poses)
v = PY.Vol((-0.5, 0.5, -0.5, 0.5, -0.5, 0.5), (512, 512, 512))
rng = np.random.default_rng(0)
S = int(sys.argv[1]) if len(sys.argv) > 1 else 10
NPK = int(sys.argv[2]) if len(sys.argv) > 2 else 40
orders = {
 "tile-order, tiles2x2x4": (lambda c, lo: (c[0]//2, c[1]//2, c[2]//4, c[0]&1, c[1]&1, c[2]&3), lambda c: (c[0]//2, c[1]//2, c[2]//4)),
 "linear-xyz, tiles2x2x4": (lambda c, lo: (c[0], c[1], c[2]), lambda c: (c[0]//2, c[1]//2, c[2]//4)),
 "linear-xyz, rows16": (lambda c, lo: (c[0], c[1], c[2]), lambda c: (c[0], c[1], c[2]//16)),
 "linear-xyz, tiles1x4x4": (lambda c, lo: (c[0], c[1], c[2]), lambda c: (c[0], c[1]//4, c[2]//4)),
 "tile-order, tiles1x4x4": (lambda c, lo: (c[0], c[1]//4, c[2]//4, c[1]&3, c[2]&3), lambda c: (c[0], c[1]//4, c[2]//4)),
 "tile-order, tiles4x4x1": (lambda c, lo: (c[0]//4, c[1]//4, c[2], c[0]&3, c[1]&3), lambda c: (c[0]//4, c[1]//4, c[2])),
}
req = {k: 0 for k in orders}
upd = 0; cellsn = 0; rounds = 0
npk = 0
while npk < NPK:
    p = int(rng.integers(0, 4))
    r0, c0 = int(rng.integers(0, H // 8)) * 8, int(rng.integers(0, W // 8)) * 8
    T = poses[p]
    O = (np.float32(T[3]), np.float32(T[7]), np.float32(T[11]))
    rays = []
    for r in range(r0, r0 + 8):
        for c in range(c0, c0 + 8):
            d = int(depth[p, r, c])
            if not (scene.DEPTH_MIN_MM <= d < scene.DEPTH_MAX_MM):
                continue
            E = PY.transform(T, PY.project_point(K, r, c, d))
            inside = v.valid_points(E) and v.valid_coords(v.get_voxel(E))
            rays.append(PY.dda_cells(v, O, E, inside)[0])
    if len(rays) < 32:
        continue
    npk += 1
    L = max(len(m) for m in rays)
    for k0 in range(0, L, S):
        cnt = {}
        for m in rays:
            for cc in m[k0:k0 + S]:
                cnt[cc] = cnt.get(cc, 0) + 1
                upd += 1
        if not cnt:
            continue
        rounds += 1
        cellsn += len(cnt)
        lo = np.array(list(cnt)).min(0)
        for name, (key, line) in orders.items():
            lst = sorted(cnt, key=lambda c: key(c, lo))
            for i in range(0, len(lst), 64):
                req[name] += len({line(c) for c in lst[i:i + 64]})
print(f"S={S} packets={NPK} rounds={rounds} updates/cell {upd/cellsn:.2f} cells/round {cellsn/rounds:.1f}")
for k in orders:
    print(f"  {k:26s} requests/update {req[k]/upd:.4f}  cells/request {cellsn/req[k]:.2f}")
