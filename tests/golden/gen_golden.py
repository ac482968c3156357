#!/usr/bin/env python3
"""Generate tests/golden/golden_v1.npz from the CPU oracle (oracle/oracle.cpp).

The reference ships no golden vectors and cannot be built here (SURVEY.md §8c,
DESIGN.md §2: parity unpinned), so these fixtures pin the oracle against regressions
and give the GPU tests a committed target.  Inputs: the analytic scene rendered at
320x240 (reference K scaled by 0.5) for two Fibonacci poses, back-projected by the
oracle (Camera.hpp:24-45); normals stored as float16 (exact inputs, widened to
float32 on load); grid [-0.5,0.5]^3 at 64^3 / 96^3 (power-of-two and non-power-of-
two deltas).  Outputs: every hot-path result.

usage: python tests/golden/gen_golden.py   (rewrites golden_v1.npz)
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [ROOT, os.path.join(ROOT, "depth-map-fusion-utils_amd")]
from dmf_amd import scene  # noqa: E402
from oracle import oracle as O  # noqa: E402

W, H = 320, 240


def inputs():
    K = scene.K_640x480.copy()
    K[[0, 2, 4, 5]] *= np.float32(0.5)
    poses = scene.fibonacci_poses(6, seed=1234)
    depth, nrm = scene.render_frames(K, W, H, poses, normals=True)
    return K, poses, depth, nrm.astype(np.float16)


def cloud(K, poses, depth, nrm16, frames=(0, 1)):
    pts, nn = [], []
    for i in frames:
        xyz = O.backproject(K, depth[i], poses[i])
        m = depth[i] > 0
        pts.append(xyz[m])
        nn.append(nrm16[i][m].astype(np.float32))
    return np.concatenate(pts), np.concatenate(nn)


def volume(n, pts, nrm):
    v = O.Volume()
    v.setDimensions(-0.5, 0.5, -0.5, 0.5, -0.5, 0.5)
    v.setVolumeSize(n, n, n)
    v.constructVolume()
    v.integratePointCloud(pts, nrm)
    return v


def compute(K, poses, depth, nrm16):
    out = {}
    pts, nn = cloud(K, poses, depth, nrm16)
    sel = np.arange(0, H * W, 97)
    xyz0 = O.backproject(K, depth[0], poses[0]).reshape(-1, 3)
    out["bp_index"] = sel.astype(np.int64)
    out["bp_xyz"] = xyz0[sel]
    ref_poses = scene.reference_style_poses(pts[::5000][:3], nn[::5000][:3], 300)
    allp = np.concatenate([poses, ref_poses]).astype(np.float32)
    out["all_poses"] = allp
    eng = O.Engine(K, H, W)
    for n in (64, 96):
        v = volume(n, pts, nn)
        out[f"occ{n}"] = v.occupied_cells_
        _, _, npts, nnrm = v.voxel_table()
        out[f"npts{n}"] = npts
        lists, found = [], []
        for T in allp:
            f, g = eng.reverseRayTraceFast(v, T, False)
            lists.append(g)
            found.append(f)
        out[f"rrtf{n}_found"] = np.array(found, np.uint8)
        out[f"rrtf{n}_counts"] = np.array([len(x) for x in lists], np.int64)
        out[f"rrtf{n}_hashes"] = np.concatenate(lists).astype(np.uint64)
        k, h = eng.forward_first_hits(v, allp[0], 10, 10, 5, 5)
        out[f"fwd{n}_k"] = k
        out[f"fwd{n}_h"] = h
        out[f"min{n}"] = np.array([eng.rayTraceAndGetMinimum(v, T) for T in allp], np.int32)
        f, g = eng.rayTraceAndGetPoints(v, allp[1])
        out[f"gp{n}"] = g
        v.reset_flags()
        out[f"zbuf{n}"] = eng.rayTraceVolume(v, allp[2])
        view, _, _, _ = v.voxel_table()
        out[f"zbuf{n}_view"] = view
        v2 = volume(n, np.zeros((0, 3), np.float32), np.zeros((0, 3), np.float32))
        hits, misses, st = O.fuse_depth(v2, K, depth, poses, dmin=200, dmax=1000)
        for name, arr in (("hits", hits), ("misses", misses)):
            nz = np.nonzero(arr)[0]
            out[f"fuse{n}_{name}_idx"] = nz.astype(np.int32)
            out[f"fuse{n}_{name}_val"] = arr[nz]
        out[f"fuse{n}_stats"] = st
        out[f"fuse{n}_logodds_sum"] = np.array([int(O.fuse_finalize(hits, misses).astype(np.int64).sum())])
    return out


def main():
    K, poses, depth, nrm16 = inputs()
    out = compute(K, poses, depth, nrm16)
    np.savez_compressed(os.path.join(HERE, "golden_v1.npz"), K=K, poses=poses, depth=depth, normals16=nrm16[:2],
                        W=np.array(W), H=np.array(H), **out)
    print("wrote", os.path.join(HERE, "golden_v1.npz"), os.path.getsize(os.path.join(HERE, "golden_v1.npz")), "bytes")


if __name__ == "__main__":
    main()
