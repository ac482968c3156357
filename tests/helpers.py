"""Shared synthetic scenes for the parity tests (SURVEY.md §8d inputs, small sizes)."""
import functools

import numpy as np

from dmf_amd import scene

K = scene.K_640x480
H, W = 480, 640
BOUNDS = (-0.5, 0.5, -0.5, 0.5, -0.5, 0.5)


@functools.lru_cache(maxsize=None)
def frames(P=6, seed=1234, width=W, height=H):
    Kx = scene.intrinsics(width, height)
    poses = scene.fibonacci_poses(P, seed=seed)
    depth, nrm = scene.render_frames(Kx, width, height, poses, normals=True)
    return poses, depth, nrm


@functools.lru_cache(maxsize=None)
def cloud(n_frames=3, P=6):
    """Back-projected depth frames (oracle back-projection) + analytic normals."""
    from oracle import oracle as O
    poses, depth, nrm = frames(P)
    pts, nn = [], []
    for i in range(n_frames):
        xyz = O.backproject(K, depth[i], poses[i])
        m = depth[i] > 0
        pts.append(xyz[m])
        nn.append(nrm[i][m])
    return np.concatenate(pts).astype(np.float32), np.concatenate(nn).astype(np.float32)


@functools.lru_cache(maxsize=None)
def ref_style_poses(n=6, seed=7):
    pts, nn = cloud()
    rng = np.random.default_rng(seed)
    idx = rng.choice(pts.shape[0], n, replace=False)
    return scene.reference_style_poses(pts[idx], nn[idx], 300)


def all_poses():
    return np.concatenate([frames()[0], ref_style_poses()])


def oracle_volume(O, n=128, bounds=BOUNDS, with_normals=True, clouds=None):
    v = O.Volume()
    v.setDimensions(*bounds)
    v.setVolumeSize(n, n, n)
    v.constructVolume()
    for pts, nn in (clouds if clouds is not None else [cloud()]):
        v.integratePointCloud(pts, nn if with_normals else None)
    return v


def gpu_volume(n=128, bounds=BOUNDS, with_normals=True, clouds=None):
    import dmf_amd
    v = dmf_amd.VoxelVolume()
    v.setDimensions(*bounds)
    v.setVolumeSize(n, n, n)
    v.constructVolume()
    for pts, nn in (clouds if clouds is not None else [cloud()]):
        v.integratePointCloud(pts, nn if with_normals else None)
    return v
