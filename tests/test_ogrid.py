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


# ---- downloadReorganizedCloud (OccupancyGrid.hpp:200-286) ----------------------------

def _adversarial_state(dims, bounds, res, seed):
    """A dense voxels_ state exercising every branch of the reorganization: centroids in
    their own voxel, in a neighbour (chains of merges), at the default (0, 0, 0) (count-0
    voxels all land in the voxel holding the origin), outside the grid and NaN; counts
    around the clean threshold (100); unoccupied voxels."""
    rng = np.random.default_rng(seed)
    n = int(np.prod(dims))
    mins = np.array(bounds[0::2], np.float64)
    res = np.asarray(res, np.float64)
    idx = np.stack(np.unravel_index(np.arange(n), dims), 1).astype(np.float64)
    own = (mins + (idx + rng.uniform(0.05, 0.95, (n, 3))) * res).astype(np.float32)
    nb = (mins + (idx + rng.integers(-1, 2, (n, 3)) + rng.uniform(0.05, 0.95, (n, 3))) * res).astype(np.float32)
    kind = rng.choice(5, n, p=[0.45, 0.3, 0.12, 0.1, 0.03])
    cen = np.where((kind == 0)[:, None], own, nb)
    cen[kind == 2] = 0.0
    cen[kind == 3] = (mins - 1.0).astype(np.float32)
    cen[kind == 4] = np.nan
    cnt = rng.choice([0, 1, 7, 99, 100, 101, 250], n).astype(np.int32)
    cnt[kind == 2] = 0
    nrm = rng.normal(size=(n, 3)).astype(np.float32)
    nrm /= np.linalg.norm(nrm, axis=1, keepdims=True).astype(np.float32)
    nrm[rng.random(n) < 0.05] = 0.0
    occ = rng.random(n) < 0.7
    fl = (occ.astype(np.uint8) | ((rng.random(n) < 0.8).astype(np.uint8) << 1))
    return nrm, cen, cnt, fl


_REORG_GRIDS = [((-0.05, 0.04, -0.035, 0.045, -0.04, 0.03), (0.01, 0.01, 0.01)),
                ((-0.031, 0.052, -0.02, 0.04, -0.05, 0.01), (0.0093, 0.0071, 0.0089))]


@pytest.mark.parametrize("grid", range(len(_REORG_GRIDS)))
@pytest.mark.parametrize("clean", [False, True])
def test_reorganized_oracle_vs_python(oracle, grid, clean):
    """The C++ restatement and an independent pure-Python one agree (adversarial states)."""
    from oracle import py_oracle as P
    bounds, res = _REORG_GRIDS[grid]
    og = _setup(oracle.OccupancyGrid(), 0, res, bounds)
    for seed in range(3):
        st = _adversarial_state(og.dims, bounds, np.float32(res), seed)
        og.set_state(*st)
        exp = P.reorganized_cloud(og.dims, bounds[0::2], np.float32(res), st[0], st[1], st[2], st[3], clean)
        got = og.downloadReorganizedCloud(clean)
        assert got.shape == exp.shape and got.shape[0] > 10
        assert np.array_equal(got.view(np.uint32), exp.view(np.uint32))


@pytest.mark.gpu
@pytest.mark.parametrize("grid", range(len(_REORG_GRIDS)))
@pytest.mark.parametrize("clean", [False, True])
def test_reorganized_gpu_adversarial(oracle, grid, clean):
    """GPU fixed-point rounds vs the sequential oracle on adversarial states, bit for bit."""
    import dmf_amd
    bounds, res = _REORG_GRIDS[grid]
    og = _setup(oracle.OccupancyGrid(), 0, res, bounds)
    gg = _setup(dmf_amd.OccupancyGrid(), 0, res, bounds)
    for seed in range(4):
        st = _adversarial_state(og.dims, bounds, np.float32(res), 100 + seed)
        og.set_state(*st)
        gg.set_state(*st)
        exp = og.downloadReorganizedCloud(clean)
        got = gg.downloadReorganizedCloud(clean)
        assert got.shape == exp.shape
        assert np.array_equal(got.view(np.uint32), exp.view(np.uint32))


@pytest.mark.gpu
@pytest.mark.parametrize("k", [0, 1])
def test_reorganized_gpu_after_update_states(oracle, k):
    """downloadReorganizedCloud after updateStates (the reference's workflow), both cleans."""
    import dmf_amd
    cloud, normals = _inputs(seed=20 + k)
    og = _setup(oracle.OccupancyGrid(), k)
    gg = _setup(dmf_amd.OccupancyGrid(), k)
    og.updateStates(cloud, normals)
    gg.updateStates(cloud, normals)
    for clean in (False, True):
        exp = og.downloadReorganizedCloud(clean)
        got = gg.downloadReorganizedCloud(clean)
        assert got.shape == exp.shape and (clean or got.shape[0] > 100)
        assert np.array_equal(got.view(np.uint32), exp.view(np.uint32))
