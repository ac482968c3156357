"""OccupancyGrid (include/OccupancyGrid.hpp:50-318): the GPU updateStates (sorted
(voxel, point) events folded per voxel in point order) reproduces the sequential-order
oracle bit for bit — normals, centroids, counts, flags and both downloads."""
import numpy as np
import pytest

import helpers as Hh


def _inputs(seed=0, n=6000):
    pts, nn = Hh.cloud()
    rng = np.random.default_rng(seed)
    idx = rng.choice(pts.shape[0], n, replace=False)
    cloud = pts[idx]
    jit = rng.normal(0, 0.0004, cloud.shape).astype(np.float32)
    normals = np.concatenate([cloud + jit, nn[idx]], axis=1).astype(np.float32)
    return cloud, normals


def _setup(G, k, res=(0.008, 0.008, 0.008), bounds=(-0.45, 0.47, -0.43, 0.44, -0.41, 0.4)):
    G.setDimensions(*bounds)
    G.setResolution(*res)
    G.setK(k)
    G.construct()
    return G


def test_ogrid_oracle_nontrivial(oracle):
    cloud, normals = _inputs()
    og = _setup(oracle.OccupancyGrid(), 1)
    og.updateStates(cloud, normals)
    nrm, cen, cnt, fl = og.state()
    assert (fl & 1).sum() > 500 and (cnt > 0).sum() > 100 and (fl & 2).sum() > (fl & 1).sum()
    assert len(og.download(0)) == (fl & 1).sum()


@pytest.mark.gpu
@pytest.mark.parametrize("k", [0, 1, 2])
def test_ogrid_parity(oracle, k):
    import dmf_amd
    cloud, normals = _inputs(seed=k)
    og = _setup(oracle.OccupancyGrid(), k)
    gg = _setup(dmf_amd.OccupancyGrid(), k)
    assert og.dims == gg.dims
    for part in (slice(0, 4000), slice(4000, None)):  # two calls: state persists
        og.updateStates(cloud[part], normals[part])
        gg.updateStates(cloud[part], normals[part])
    for a, b in zip(og.state(), gg.state()):
        assert np.array_equal(a.view(np.uint8), b.view(np.uint8))
    assert np.array_equal(og.download(0), gg.downloadCloud())
    assert np.array_equal(og.download(1), gg.downloadHQCloud())


@pytest.mark.gpu
def test_ogrid_non_pow2_and_outside_points(oracle):
    import dmf_amd
    cloud, normals = _inputs(seed=7, n=3000)
    cloud = np.concatenate([cloud, np.array([[5.0, 5.0, 5.0], [-0.449, 0.0, 0.0]], np.float32)])
    normals = np.concatenate([normals, np.array([[5, 5, 5, 0, 0, 1], [-0.449, 0, 0, 1, 0, 0]], np.float32)])
    res = (0.0071, 0.0093, 0.0067)
    og = _setup(oracle.OccupancyGrid(), 1, res)
    gg = _setup(dmf_amd.OccupancyGrid(), 1, res)
    og.updateStates(cloud, normals)
    gg.updateStates(cloud, normals)
    for a, b in zip(og.state(), gg.state()):
        assert np.array_equal(a.view(np.uint8), b.view(np.uint8))
