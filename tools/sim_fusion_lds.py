#!/usr/bin/env python3
"""CPU model: LDS bank cycles of the fusion replay's ds_add for several replay orders.

Per replay step (one wave instruction), each 32-lane group costs max over banks
((word address) mod 32) of the lanes on that bank (same-address atomics serialise);
the linear box layout of k_fuse_l is used.  Neighbouring rays of an 8x8 packet sit
in the same cell at the same step, so the order in which each lane replays its cells
decides the conflicts.  usage: tools/sim_fusion_lds.py [S] [packets]
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
NPK = int(sys.argv[2]) if len(sys.argv) > 2 else 30

def cycles(addrs):
    # addrs: list of (lane, word) active; 2 groups of 32 lanes, bank = word % 32; every lane on a bank costs a cycle
    tot = 0
    for g in (0, 1):
        cnt = {}
        for l, a in addrs:
            if (l >> 5) == g:
                cnt[a % 32] = cnt.get(a % 32, 0) + 1
        tot += max(cnt.values()) if cnt else 0
    return tot

def order_fwd(l, n): return list(range(n))
def order_bwd_odd(l, n): return list(range(n))[::-1] if l & 1 else list(range(n))
def order_rot(l, n):
    if n == 0: return []
    o = (l * 3 + (l >> 3) * 5) % n
    return [(o + k) % n for k in range(n)]
def order_rot2(l, n):
    if n == 0: return []
    o = ((l & 7) + 2 * (l >> 3)) % n
    r = [(o + k) % n for k in range(n)]
    return r[::-1] if l & 1 else r
ORD = {"forward": order_fwd, "odd-backward (current)": order_bwd_odd, "rotated": order_rot, "rotated+odd-back": order_rot2}
res = {k: 0 for k in ORD}; ideal = 0; inst = 0
npk = 0
while npk < NPK:
    p = int(rng.integers(0, 4))
    r0, c0 = int(rng.integers(0, H // 8)) * 8, int(rng.integers(0, W // 8)) * 8
    T = poses[p]
    O = (np.float32(T[3]), np.float32(T[7]), np.float32(T[11]))
    rays = [[] for _ in range(64)]
    ok = 0
    for r in range(r0, r0 + 8):
        for c in range(c0, c0 + 8):
            l = (r - r0) * 8 + (c - c0)
            d = int(depth[p, r, c])
            if not (scene.DEPTH_MIN_MM <= d < scene.DEPTH_MAX_MM):
                continue
            E = PY.transform(T, PY.project_point(K, r, c, d))
            inside = v.valid_points(E) and v.valid_coords(v.get_voxel(E))
            rays[l] = PY.dda_cells(v, O, E, inside)[0]
            ok += 1
    if ok < 32:
        continue
    npk += 1
    L = max(len(m) for m in rays)
    for k0 in range(0, L, S):
        segs = [m[k0:k0 + S] for m in rays]
        cells = [c for sg in segs for c in sg]
        if not cells:
            continue
        a = np.array(cells); lo = a.min(0); hi = a.max(0); dim = hi - lo + 1
        lin = lambda c: ((c[0] - lo[0]) * dim[1] + (c[1] - lo[1])) * dim[2] + (c[2] - lo[2])
        for name, f in ORD.items():
            ords = [f(l, len(segs[l])) for l in range(64)]
            for k in range(S):
                addrs = [(l, lin(segs[l][ords[l][k]])) for l in range(64) if k < len(segs[l])]
                if addrs:
                    res[name] += cycles(addrs)
        for k in range(S):
            n = sum(1 for l in range(64) if k < len(segs[l]))
            if n:
                ideal += (1 if any(k < len(segs[l]) for l in range(32)) else 0) + (1 if any(k < len(segs[l]) for l in range(32, 64)) else 0)
                inst += 1
print(f"S={S} instructions {inst}  conflict-free cycles {ideal}")
for k in ORD:
    print(f"  {k:24s} LDS cycles {res[k]}  x{res[k]/ideal:.2f}")
