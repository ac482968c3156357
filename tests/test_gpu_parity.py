"""GPU parity: every hot-path entry point through the C ABI vs the CPU oracle.

Bit-exact for every integer/index output (occupied_cells_ order, flags, lists,
first hits, z-buffer, counters) and for the back-projected float coordinates
(north_star tolerance is 1e-5; the fp64 + no-FMA restatement is exact, so the
test demands equality of the float32 bit patterns).
"""
import numpy as np
import pytest

import helpers as Hh
from helpers import H, K, W

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dmf():
    import dmf_amd
    return dmf_amd


@pytest.fixture(scope="module")
def cam(dmf):
    return dmf.Camera(K, H, W)


@pytest.fixture(scope="module")
def engine(dmf, cam):
    return dmf.RayTracingEngine(cam)


@pytest.fixture(scope="module")
def oeng(oracle):
    return oracle.Engine(K, H, W)


def test_backproject_bitexact(oracle, engine):
    poses, depth, _ = Hh.frames()
    vol = Hh.gpu_volume(clouds=[])
    for i in range(3):
        g = engine.backproject(vol, depth[i], poses[i])
        o = oracle.backproject(K, depth[i], poses[i])
        assert np.array_equal(g.view(np.uint32), o.view(np.uint32))
        assert np.max(np.abs(g - o)) <= 1e-5


def test_backproject_non_orthonormal(oracle, engine):
    _, depth, _ = Hh.frames()
    T = Hh.ref_style_poses()[0]
    vol = Hh.gpu_volume(clouds=[])
    g = engine.backproject(vol, depth[0], T)
    o = oracle.backproject(K, depth[0], T)
    assert np.array_equal(g.view(np.uint32), o.view(np.uint32))


@pytest.mark.parametrize("with_normals", [True, False])
def test_integrate_parity(oracle, with_normals):
    pts, nn = Hh.cloud()
    half = pts.shape[0] // 2
    clouds = [(pts[:half], nn[:half]), (pts[half:], nn[half:])]
    ov = Hh.oracle_volume(oracle, with_normals=with_normals, clouds=clouds)
    gv = Hh.gpu_volume(with_normals=with_normals, clouds=clouds)
    assert np.array_equal(ov.occupied_cells_, gv.occupied_cells_)
    assert np.array_equal(ov.occupancy_dense(), gv.occupancy_dense())
    _, _, onp, onn = ov.voxel_table()
    gnp, gnn = gv.voxel_counts()
    assert np.array_equal(onp, gnp) and np.array_equal(onn, gnn)
    occ = ov.occupied_cells_
    for h in occ[:: max(1, len(occ) // 50)]:
        x, y, z = int(h) >> 40, (int(h) >> 20) & 0xFFFFF, int(h) & 0xFFFFF
        op, on = ov.voxel_points(x, y, z)
        gp, gn = gv.voxel_points(h)
        assert np.array_equal(op, gp)
        if with_normals:
            assert np.array_equal(on, gn)
    assert gv.info()["num_points"] == int(onp.sum())


def test_integrate_points_outside_and_empty(oracle, dmf):
    gv = Hh.gpu_volume(clouds=[])
    gv.integratePointCloud(np.zeros((0, 3), np.float32))
    assert len(gv.occupied_cells_) == 0
    pts = np.array([[0.6, 0, 0], [-0.5, 0, 0], [0.1, 0.1, 0.1], [0.1, 0.1, 0.1001], [0.49999, 0, 0]], np.float32)
    nn = np.tile(np.array([[0, 0, 1]], np.float32), (5, 1))
    ov = Hh.oracle_volume(oracle, clouds=[(pts, nn)])
    gv.integratePointCloud(pts, nn)
    assert np.array_equal(ov.occupied_cells_, gv.occupied_cells_)


def _flags(v_or, v_gpu):
    ov, og, _, _ = v_or.voxel_table()
    gview, ggood = v_gpu.voxel_flags()
    return ov, og, gview, ggood


@pytest.mark.parametrize("kernel", [0, 4, 5, 3, 1, 2])
def test_reverse_fast_parity(oracle, engine, oeng, kernel):
    """reverseRayTraceFast (RayTracingEngine.hpp:136-226) over 12 poses, every march kernel
    (DMF_KNOB_REVERSE_KERNEL): 0 = the default work queue in spatial (Morton) item order with
    the item -> slot mask permutation, its workgroup units taken from per-XCD queues with work
    stealing (k_reverse_x), 4 = the same with per-wave units, 5 = the spatial-order queue on a
    (chunk, pose) grid (k_reverse_q), 3 = the work queue in occupied_cells_ order, 1 / 2 =
    one lane per (voxel, pose) without / with brick skipping: lists (order included), found
    and view / good flags equal the oracle's."""
    from dmf_amd import _lib
    ov = Hh.oracle_volume(oracle)
    gv = Hh.gpu_volume()
    _lib.set_knob(gv, "reverse_kernel", kernel)
    poses = Hh.all_poses()
    found, lists = engine.reverseRayTraceFastBatch(gv, poses, viz=False)
    for i, T in enumerate(poses):
        f, g = oeng.reverseRayTraceFast(ov, T, False)
        assert f == bool(found[i])
        assert np.array_equal(g, lists[i]), f"pose {i}: {len(g)} vs {len(lists[i])}"
    # viz=True flags, single-pose reference signature
    ov.reset_flags()
    gv.reset_flags()
    for T in poses[:4]:
        f, g = oeng.reverseRayTraceFast(ov, T, True)
        f2, g2 = engine.reverseRayTraceFast(gv, T, True)
        assert f == f2 and np.array_equal(g, g2)
    a, b, c, d = _flags(ov, gv)
    assert np.array_equal(a, c) and np.array_equal(b, d)
    assert sum(len(x) for x in lists) > 0


def test_reverse_full_parity(oracle, engine, oeng):
    ov = Hh.oracle_volume(oracle, n=64)
    gv = Hh.gpu_volume(n=64)
    for T in Hh.all_poses()[:6]:
        f, g = oeng.reverseRayTrace(ov, T, True)
        f2, g2 = engine.reverseRayTrace(gv, T, True)
        assert f == f2 and np.array_equal(g, g2)
    a, b, c, d = _flags(ov, gv)
    assert np.array_equal(a, c) and np.array_equal(b, d)


@pytest.mark.parametrize("cap", [0, 1, 2, 255])
def test_reverse_sparse_partial_bricks(oracle, engine, oeng, cap):
    """Empty-space skipping stress: a sparse scatter of occupied cells in a grid whose
    dims are not multiples of the 8-cell brick and whose deltas are not powers of two;
    cameras outside and inside the volume; the brick distance field saturated at the default
    (63), 1, 2 and 255 bricks (DMF_KNOB_BDIST_CAP: cubes of one brick up to cubes reaching past
    the volume's faces, whose jumps may leave the volume at once).  Lists and view/good flags
    must be exact."""
    rng = np.random.default_rng(21)
    bounds = (-0.45, 0.52, -0.4, 0.47, -0.33, 0.41)
    dims = (91, 77, 61)
    pts = rng.uniform([-0.44, -0.39, -0.32], [0.51, 0.46, 0.40], (400, 3)).astype(np.float32)
    nn = rng.normal(size=(400, 3)).astype(np.float32)
    nn /= np.linalg.norm(nn, axis=1, keepdims=True)
    ov = oracle.Volume()
    ov.setDimensions(*bounds)
    ov.setVolumeSize(*dims)
    ov.constructVolume()
    ov.integratePointCloud(pts, nn)
    import dmf_amd
    gv = dmf_amd.VoxelVolume()
    gv.setDimensions(*bounds)
    gv.setVolumeSize(*dims)
    gv.constructVolume()
    from dmf_amd import _lib
    _lib.set_knob(gv, "bdist_cap", cap)
    gv.integratePointCloud(pts, nn)
    assert np.array_equal(ov.occupied_cells_, gv.occupied_cells_)
    from dmf_amd import scene
    poses = np.concatenate([scene.fibonacci_poses(10, seed=5), scene.reference_style_poses(pts[:6], nn[:6], 150)])
    found, lists = engine.reverseRayTraceFastBatch(gv, poses, viz=False)
    total = 0
    for i, T in enumerate(poses):
        f, g = oeng.reverseRayTraceFast(ov, T, False)
        assert f == bool(found[i]) and np.array_equal(g, lists[i]), f"pose {i}"
        total += len(g)
    assert total > 0
    for T in poses[:5]:
        f, g = oeng.reverseRayTraceFast(ov, T, True)
        f2, g2 = engine.reverseRayTraceFast(gv, T, True)
        assert f == f2 and np.array_equal(g, g2)
    for T in poses[-3:]:
        f, g = oeng.reverseRayTrace(ov, T, True)
        f2, g2 = engine.reverseRayTrace(gv, T, True)
        assert f == f2 and np.array_equal(g, g2)
    a, b, c, d = _flags(ov, gv)
    assert np.array_equal(a, c) and np.array_equal(b, d)


@pytest.mark.parametrize("zstart,zdelta,stride", [(10, 10, 5), (5, 1, 10), (10, 3, 1)])
def test_forward_first_hits(oracle, engine, oeng, zstart, zdelta, stride):
    ov = Hh.oracle_volume(oracle)
    gv = Hh.gpu_volume()
    for T in Hh.all_poses()[:5]:
        ko, ho = oeng.forward_first_hits(ov, T, zstart, zdelta, stride, stride)
        kg, hg = engine.forward_first_hits(gv, T, zstart, zdelta, stride, stride)
        assert np.array_equal(ko, kg)
        assert np.array_equal(ho[ko >= 0], hg[kg >= 0])


@pytest.mark.parametrize("sparse", [True, False])
def test_forward_family(oracle, engine, oeng, sparse):
    ov = Hh.oracle_volume(oracle)
    gv = Hh.gpu_volume()
    for T in Hh.all_poses()[:4]:
        assert oeng.rayTraceAndGetMinimum(ov, T, 1, sparse) == engine.rayTraceAndGetMinimum(gv, T, 1, sparse)
        f, g = oeng.rayTraceAndGetPoints(ov, T, 10, sparse)
        f2, g2 = engine.rayTraceAndGetPoints(gv, T, 10, sparse)
        assert f == f2 and np.array_equal(g, g2)
        f, g = oeng.rayTraceAndGetGoodPoints(ov, T, 10, sparse)
        f2, g2 = engine.rayTraceAndGetGoodPoints(gv, T, 10, sparse)
        assert f == f2 and np.array_equal(g, g2)
    ov.reset_flags()
    gv.reset_flags()
    for i, T in enumerate(Hh.all_poses()[:4]):
        oeng.rayTraceAndClassify(ov, T, 10, i + 2, sparse)
        engine.rayTraceAndClassify(gv, T, 10, i + 2, sparse)
    a, b, c, d = _flags(ov, gv)
    assert np.array_equal(a, c) and np.array_equal(b, d)
    ov.reset_flags()
    gv.reset_flags()
    for T in Hh.all_poses()[4:8]:
        oeng.rayTrace(ov, T, 10, sparse)
        engine.rayTrace(gv, T, 10, sparse)
    a, b, c, d = _flags(ov, gv)
    assert np.array_equal(a, c) and np.array_equal(b, d)


def test_ray_trace_volume(oracle, engine, oeng):
    ov = Hh.oracle_volume(oracle, n=64)
    gv = Hh.gpu_volume(n=64)
    for T in Hh.all_poses()[:4]:
        assert np.array_equal(oeng.rayTraceVolume(ov, T), engine.rayTraceVolume(gv, T))
    a, b, c, d = _flags(ov, gv)
    assert np.array_equal(a, c)


def test_will_collide(oracle, dmf):
    ov = Hh.oracle_volume(oracle)
    gv = Hh.gpu_volume()
    P = Hh.all_poses().reshape(-1, 3, 4)[:, :, 3]
    a = np.repeat(P, len(P), axis=0)
    b = np.tile(P, (len(P), 1))
    g = dmf.will_collide(gv, a, b)
    o = np.array([oracle.will_collide(ov, a[i], b[i]) for i in range(len(a))])
    assert np.array_equal(g, o)
    assert g.any() and not g.all()


def test_collision_cost_map(oracle, dmf):
    """Planner::run_tsp cost map (tests/CameraPathGen.cpp:310-331) over V*V pairs."""
    ov = Hh.oracle_volume(oracle)
    gv = Hh.gpu_volume()
    poses = Hh.all_poses().reshape(-1, 12)
    # add centres inside the box (every segment between them crosses the surface) and a
    # duplicate centre (zero-length segment -> cost 0, no collision)
    rng = np.random.default_rng(7)
    inner = np.tile(poses[:1], (6, 1))
    lo, hi = np.array(Hh.BOUNDS[0::2]), np.array(Hh.BOUNDS[1::2])
    inner[:, 3::4] = (lo + (hi - lo) * rng.uniform(0.2, 0.8, (6, 3))).astype(np.float32)
    poses = np.concatenate([poses, inner, poses[:1]])
    got = dmf.collision_cost_map(gv, poses)
    exp = oracle.collision_cost_map(ov, poses)
    assert np.array_equal(got, exp)
    coll = got == np.iinfo(np.int32).max
    assert coll.any() and not coll.all()
    assert np.all(np.diag(got) == 0) and got[0, -1] == 0
    # the same pairs through the segment-batched willCollide
    V = len(poses)
    c = poses[:, 3::4]
    wc = dmf.will_collide(gv, np.repeat(c, V, axis=0), np.tile(c, (V, 1))).reshape(V, V)
    assert np.array_equal(wc, coll)
    # edge sizes
    assert dmf.collision_cost_map(gv, poses[:0]).shape == (0, 0)
    assert np.array_equal(dmf.collision_cost_map(gv, poses[:1]), np.zeros((1, 1), np.int32))


def test_collision_cost_map_sparse(oracle, dmf):
    """The cost map over a sparse scatter in a grid whose dims are not multiples of the brick and
    whose deltas are not powers of two, with centres inside and outside the volume: equal to the
    oracle's sequential willCollide."""
    import dmf_amd
    rng = np.random.default_rng(29)
    bounds = (-0.45, 0.52, -0.4, 0.47, -0.33, 0.41)
    dims = (91, 77, 61)
    pts = rng.uniform([-0.44, -0.39, -0.32], [0.51, 0.46, 0.40], (150, 3)).astype(np.float32)
    nn = np.tile(np.array([[0, 0, 1]], np.float32), (150, 1))
    ov = oracle.Volume()
    ov.setDimensions(*bounds)
    ov.setVolumeSize(*dims)
    ov.constructVolume()
    ov.integratePointCloud(pts, nn)
    gv = dmf_amd.VoxelVolume()
    gv.setDimensions(*bounds)
    gv.setVolumeSize(*dims)
    gv.constructVolume()
    gv.integratePointCloud(pts, nn)
    V = 48
    poses = np.tile(np.eye(3, 4, dtype=np.float32).reshape(1, 12), (V, 1))
    lo, hi = np.array(bounds[0::2]), np.array(bounds[1::2])
    poses[:, 3::4] = (lo + (hi - lo) * rng.uniform(-0.1, 1.1, (V, 3))).astype(np.float32)
    got = dmf.collision_cost_map(gv, poses)
    exp = oracle.collision_cost_map(ov, poses)
    assert np.array_equal(got, exp)
    coll = got == np.iinfo(np.int32).max
    assert coll.any() and not coll.all()


def test_collision_cost_map_device_invalid_centre(dmf):
    import ctypes as C
    import torch
    gv = Hh.gpu_volume()
    poses = Hh.all_poses().reshape(-1, 12)[:4].copy()
    poses[2, 3] = np.nan
    with pytest.raises(dmf.DmfError):
        dmf.collision_cost_map(gv, poses)
    dp = torch.from_numpy(poses).cuda()
    dm = torch.zeros((4, 4), dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()
    gv._L.dmf_volume_set_stream(gv._h, C.c_void_p(torch.cuda.current_stream().cuda_stream))
    assert gv._L.dmf_collision_cost_map_device(gv._h, C.c_void_p(dp.data_ptr()), 4, C.c_void_p(dm.data_ptr())) == 0
    torch.cuda.synchronize()
    m = dm.cpu().numpy()
    assert (m[2, :] == -1).all() and (m[:, 2] == -1).all()
    ok = np.delete(np.delete(m, 2, 0), 2, 1)
    assert np.array_equal(ok, dmf.collision_cost_map(gv, np.delete(poses, 2, 0)))


def test_fuse_parity(oracle, engine):
    poses, depth, _ = Hh.frames()
    ov = Hh.oracle_volume(oracle, clouds=[])
    gv = Hh.gpu_volume(clouds=[])
    ho, mo, so = oracle.fuse_depth(ov, K, depth, poses, dmin=200, dmax=1000)
    import dmf_amd
    prm = dmf_amd.FuseParams(dmin_mm=200, dmax_mm=1000)
    hg, mg, sg = engine.fuse_depth(gv, depth, poses, prm)
    assert np.array_equal(so, sg)
    assert np.array_equal(ho, hg) and np.array_equal(mo, mg)
    assert np.array_equal(oracle.fuse_finalize(ho, mo), engine.fuse_finalize(gv, hg, mg))


def test_fuse_device_tiled_counters(oracle, engine, dmf):
    """Device form: tiled counters (accumulated over two calls) -> linear via
    dmf_fuse_counters_to_linear_device, and dmf_fuse_finalize_device from the tiled
    counters, equal the oracle.  Odd dims exercise the padded tiles."""
    import ctypes as C
    from dmf_amd import _lib
    poses, depth, _ = Hh.frames()
    dims = (61, 50, 47)
    ov = oracle.Volume()
    ov.setDimensions(*Hh.BOUNDS)
    ov.setVolumeSize(*dims)
    ov.constructVolume()
    ho, mo, _ = oracle.fuse_depth(ov, K, depth, poses, dmin=200, dmax=1000)
    gv = dmf.VoxelVolume()
    gv.setDimensions(*Hh.BOUNDS)
    gv.setVolumeSize(*dims)
    gv.constructVolume()
    L, h = gv._L, gv._h
    ncell = int(np.prod(gv.dims))
    nt = C.c_int64()
    _lib.check(L.dmf_fuse_counter_cells(h, C.addressof(nt)))
    nt = nt.value
    assert nt >= ncell and nt % 16 == 0

    def dmalloc(nbytes):
        p = C.c_void_p()
        _lib.check(L.dmf_device_malloc(h, C.addressof(p), nbytes))
        return p.value

    dd, dp, dh, dm, dl, dlo = (dmalloc(b) for b in (depth.nbytes, poses.astype(np.float32).nbytes, 4 * nt, 4 * nt,
                                                     4 * ncell, 2 * ncell))
    try:
        d16 = np.ascontiguousarray(depth, np.uint16)
        p32 = np.ascontiguousarray(poses, np.float32)
        _lib.check(L.dmf_memcpy_h2d(h, dd, d16.ctypes.data, d16.nbytes))
        _lib.check(L.dmf_memcpy_h2d(h, dp, p32.ctypes.data, p32.nbytes))
        _lib.check(L.dmf_memset_device(h, dh, 0, 4 * nt))
        _lib.check(L.dmf_memset_device(h, dm, 0, 4 * nt))
        prm = dmf.FuseParams(dmin_mm=200, dmax_mm=1000)
        cam = _lib.make_camera(K, H, W)
        P = len(poses)
        half = P // 2
        _lib.check(L.dmf_fuse_depth_device(h, C.addressof(cam), dd, dp, half, C.addressof(prm), dh, dm, None))
        _lib.check(L.dmf_fuse_depth_device(h, C.addressof(cam), dd + d16[0].nbytes * half, dp + 48 * half, P - half,
                                           C.addressof(prm), dh, dm, None))
        out = {}
        for name, src in (("hits", dh), ("misses", dm)):
            a = np.zeros(ncell, np.int32)
            _lib.check(L.dmf_fuse_counters_to_linear_device(h, src, dl))
            _lib.check(L.dmf_memcpy_d2h(h, a.ctypes.data, dl, 4 * ncell))
            out[name] = a
        assert np.array_equal(out["hits"], ho) and np.array_equal(out["misses"], mo)
        lg = np.zeros(ncell, np.int16)
        _lib.check(L.dmf_fuse_finalize_device(h, dh, dm, C.addressof(prm), dlo))
        _lib.check(L.dmf_memcpy_d2h(h, lg.ctypes.data, dlo, 2 * ncell))
        assert np.array_equal(lg, oracle.fuse_finalize(ho, mo))
    finally:
        for p in (dd, dp, dh, dm, dl, dlo):
            L.dmf_device_free(h, p)


def test_fuse_non_orthonormal_and_inside_cameras(oracle, engine):
    _, depth, _ = Hh.frames()
    poses = Hh.ref_style_poses()[:3]  # cameras 0.3 m from the surface: inside the grid
    ov = Hh.oracle_volume(oracle, n=100, clouds=[])  # non power-of-two delta path
    gv = Hh.gpu_volume(n=100, clouds=[])
    ho, mo, so = oracle.fuse_depth(ov, K, depth[:3], poses)
    hg, mg, sg = engine.fuse_depth(gv, depth[:3], poses)
    assert np.array_equal(so, sg) and np.array_equal(ho, hg) and np.array_equal(mo, mg)


def test_truncated_dims_and_odd_bounds(oracle, engine, oeng):
    # float bounds from a cloud's min/max: constructVolume may truncate dims (Volume.hpp:121-123)
    pts, nn = Hh.cloud()
    lo, hi = pts.min(0), pts.max(0)
    bounds = (float(lo[0]), float(hi[0]), float(lo[1]), float(hi[1]), float(lo[2]), float(hi[2]))
    n = [int((hi[i] - lo[i]) * 125) for i in range(3)]
    ov = oracle.Volume()
    ov.setDimensions(*bounds)
    ov.setVolumeSize(*n)
    ov.constructVolume()
    ov.integratePointCloud(pts, nn)
    import dmf_amd
    gv = dmf_amd.VoxelVolume()
    gv.setDimensions(*bounds)
    gv.setVolumeSize(*n)
    gv.constructVolume()
    gv.integratePointCloud(pts, nn)
    assert ov.dims == gv.dims
    assert np.array_equal(ov.occupied_cells_, gv.occupied_cells_)
    for T in Hh.all_poses()[:3]:
        f, g = oeng.reverseRayTraceFast(ov, T, False)
        f2, g2 = engine.reverseRayTraceFast(gv, T, False)
        assert f == f2 and np.array_equal(g, g2)


def test_errors_are_loud(dmf, engine):
    gv = Hh.gpu_volume(clouds=[])
    with pytest.raises(dmf.DmfError):
        engine.rayTraceAndGetMinimum(gv, Hh.frames()[0][0], 0, True)  # zdelta 0: reference never ends
    v = dmf.VoxelVolume()
    with pytest.raises(dmf.DmfError):
        v.integratePointCloud(np.zeros((4, 3), np.float32))  # not constructed


def test_fuse_kernel_repeatable(oracle, engine):
    """Counts are exact integers: every repetition must reproduce the oracle exactly
    (guards the LDS aggregation rounds against races)."""
    _, depth, _ = Hh.frames()
    poses = np.concatenate([Hh.ref_style_poses()[:2], Hh.frames()[0][:2]])
    frames = np.concatenate([depth[:2], depth[2:4]])
    ov = Hh.oracle_volume(oracle, n=96, clouds=[])
    ho, mo, so = oracle.fuse_depth(ov, K, frames, poses)
    gv = Hh.gpu_volume(n=96, clouds=[])
    for _ in range(5):
        hg, mg, sg = engine.fuse_depth(gv, frames, poses)
        assert np.array_equal(so, sg) and np.array_equal(ho, hg) and np.array_equal(mo, mg)


def test_golden_fixture_gpu(dmf):
    """GPU results against the committed golden vectors (tests/golden/gen_golden.py)."""
    import os
    z = np.load(os.path.join(os.path.dirname(__file__), "golden", "golden_v1.npz"))
    K, poses, depth = z["K"], z["poses"], z["depth"]
    W, H = int(z["W"]), int(z["H"])
    cam = dmf.Camera(K, H, W)
    eng = dmf.RayTracingEngine(cam)
    pts, nn = [], []
    vol0 = dmf.VoxelVolume()
    vol0.setDimensions(-0.5, 0.5, -0.5, 0.5, -0.5, 0.5)
    vol0.setVolumeSize(8, 8, 8)
    vol0.constructVolume()
    for i in (0, 1):
        xyz = eng.backproject(vol0, depth[i], poses[i])
        if i == 0:
            assert np.array_equal(xyz.reshape(-1, 3)[z["bp_index"]].view(np.uint32), z["bp_xyz"].view(np.uint32))
        m = depth[i] > 0
        pts.append(xyz[m])
        nn.append(z["normals16"][i][m].astype(np.float32))
    pts, nn = np.concatenate(pts), np.concatenate(nn)
    allp = z["all_poses"]
    for n in (64, 96):
        v = dmf.VoxelVolume()
        v.setDimensions(-0.5, 0.5, -0.5, 0.5, -0.5, 0.5)
        v.setVolumeSize(n, n, n)
        v.constructVolume()
        v.integratePointCloud(pts, nn)
        assert np.array_equal(v.occupied_cells_, z[f"occ{n}"])
        assert np.array_equal(v.voxel_counts()[0], z[f"npts{n}"])
        found, lists = eng.reverseRayTraceFastBatch(v, allp, viz=False)
        assert np.array_equal(found.astype(np.uint8), z[f"rrtf{n}_found"])
        assert np.array_equal(np.array([len(x) for x in lists]), z[f"rrtf{n}_counts"])
        assert np.array_equal(np.concatenate(lists), z[f"rrtf{n}_hashes"])
        k, h = eng.forward_first_hits(v, allp[0], 10, 10, 5, 5)
        assert np.array_equal(k, z[f"fwd{n}_k"]) and np.array_equal(h[k >= 0], z[f"fwd{n}_h"][k >= 0])
        assert np.array_equal(np.array([eng.rayTraceAndGetMinimum(v, T) for T in allp], np.int32), z[f"min{n}"])
        assert np.array_equal(eng.rayTraceAndGetPoints(v, allp[1])[1], z[f"gp{n}"])
        v.reset_flags()
        assert np.array_equal(eng.rayTraceVolume(v, allp[2]), z[f"zbuf{n}"])
        assert np.array_equal(v.voxel_flags()[0], z[f"zbuf{n}_view"])
        f = dmf.VoxelVolume()
        f.setDimensions(-0.5, 0.5, -0.5, 0.5, -0.5, 0.5)
        f.setVolumeSize(n, n, n)
        f.constructVolume()
        hits, misses, st = eng.fuse_depth(f, depth, poses, dmf.FuseParams(dmin_mm=200, dmax_mm=1000))
        assert np.array_equal(st, z[f"fuse{n}_stats"])
        for name, arr in (("hits", hits), ("misses", misses)):
            nz = np.nonzero(arr)[0]
            assert np.array_equal(nz, z[f"fuse{n}_{name}_idx"]) and np.array_equal(arr[nz], z[f"fuse{n}_{name}_val"])
        L = eng.fuse_finalize(f, hits, misses)
        assert int(L.astype(np.int64).sum()) == int(z[f"fuse{n}_logodds_sum"][0])


def test_greedy_set_cover(oracle, engine, oeng, dmf):
    """Algorithms.hpp:38-86 greedySetCover over the reverseRayTraceFast good sets of all
    candidate poses (tests/SetCover.cpp:218-240) == oracle restatement (std::set_difference)."""
    ov = Hh.oracle_volume(oracle)
    gv = Hh.gpu_volume()
    from dmf_amd import scene
    poses = np.concatenate([Hh.all_poses(), scene.fibonacci_poses(20, seed=77)])
    sets = [oeng.reverseRayTraceFast(ov, T, False)[1] for T in poses]
    for min_gain in (5, 1, 200):
        exp = oracle.greedy_set_cover(sets, min_gain)
        got = engine.setCover(gv, poses, min_gain)
        assert np.array_equal(exp, got), (min_gain, exp, got)
    assert len(oracle.greedy_set_cover(sets, 5)) >= 2
    # device-mask form over the same good sets
    import ctypes as C
    from dmf_amd import _lib
    L, h = gv._L, gv._h
    P = len(poses)
    V = len(gv.occupied_cells_)
    words = (V + 63) // 64
    masks = np.zeros((P, words), np.uint64)
    slot = {int(x): i for i, x in enumerate(gv.occupied_cells_)}
    for p, st in enumerate(sets):
        for x in st:
            i = slot[int(x)]
            masks[p, i // 64] |= np.uint64(1) << np.uint64(i % 64)
    d = C.c_void_p()
    _lib.check(L.dmf_device_malloc(h, C.addressof(d), masks.nbytes))
    try:
        _lib.check(L.dmf_memcpy_h2d(h, d.value, masks.ctypes.data, masks.nbytes))
        sel = np.zeros(P, np.int32)
        n = C.c_int32()
        _lib.check(L.dmf_greedy_set_cover_masks_device(h, d.value, P, words, 5, sel.ctypes.data, C.addressof(n)))
        assert np.array_equal(sel[:n.value], oracle.greedy_set_cover(sets, 5))
    finally:
        L.dmf_device_free(h, d.value)


def test_golden_config1_gpu(dmf):
    """SURVEY.md §8c-3 config 1 (tests/Raytracing.cpp:61-92 sequence, 640x480, one pose)
    against tests/golden/golden_config1.npz (gen_golden_config1.py)."""
    import hashlib
    import os
    z = np.load(os.path.join(os.path.dirname(__file__), "golden", "golden_config1.npz"))
    sha = lambda a: np.frombuffer(hashlib.sha256(np.ascontiguousarray(a).tobytes()).digest(), np.uint8)
    K, pose, depth, q = z["K"], z["pose"], z["depth"], z["normals_q"]
    eng = dmf.RayTracingEngine(dmf.Camera(K, 480, 640))
    v0 = dmf.VoxelVolume()
    v0.setDimensions(-0.5, 0.5, -0.5, 0.5, -0.5, 0.5)
    v0.setVolumeSize(8, 8, 8)
    v0.constructVolume()
    xyz = eng.backproject(v0, depth, pose)
    assert np.array_equal(sha(xyz), z["bp_sha"])
    m = depth > 0
    pts = xyz[m]
    nrm = (q[m].astype(np.float32) / np.float32(127.0)).astype(np.float32)
    lo, hi = pts.min(0), pts.max(0)
    v = dmf.VoxelVolume()
    v.setDimensions(float(lo[0]), float(hi[0]), float(lo[1]), float(hi[1]), float(lo[2]), float(hi[2]))
    v.setVolumeSize(*[int(np.float32(hi[i] - lo[i]) * np.float32(125)) for i in range(3)])
    v.constructVolume()
    v.integratePointCloud(pts, nrm)
    assert tuple(v.dims) == tuple(z["dims"])
    assert np.array_equal(v.occupied_cells_, z["occ"])
    assert np.array_equal(sha(v.voxel_counts()[0].astype(np.int64)), z["npts_sha"])
    found, good = eng.reverseRayTraceFast(v, pose, True)
    assert int(found) == int(z["rrtf_found"][0]) and np.array_equal(good, z["rrtf_good"])
    view, goodf = v.voxel_flags()
    assert np.array_equal(sha(view.astype(np.int32)), z["rrtf_view_sha"])
    assert np.array_equal(sha(goodf.astype(np.uint8)), z["rrtf_goodf_sha"])
    k, h = eng.forward_first_hits(v, pose, 10, 10, 1, 1)
    assert np.array_equal(sha(k), z["fwd_k_sha"]) and np.array_equal(sha(h), z["fwd_h_sha"])
    assert eng.rayTraceAndGetMinimum(v, pose) == int(z["minimum"][0])
    vf = dmf.VoxelVolume()
    vf.setDimensions(-0.5, 0.5, -0.5, 0.5, -0.5, 0.5)
    vf.setVolumeSize(128, 128, 128)
    vf.constructVolume()
    from dmf_amd import scene
    hits, misses, st = eng.fuse_depth(vf, depth[None], pose[None],
                                      dmf.FuseParams(dmin_mm=scene.DEPTH_MIN_MM, dmax_mm=scene.DEPTH_MAX_MM))
    assert np.array_equal(st, z["fuse_stats"])
    assert np.array_equal(sha(hits), z["fuse_hits_sha"]) and np.array_equal(sha(misses), z["fuse_misses_sha"])
    assert np.array_equal(sha(eng.fuse_finalize(vf, hits, misses)), z["fuse_logodds_sha"])


@pytest.mark.parametrize("fwd_kernel", [0, 1, 2])
def test_forward_first_hits_batched_device(oracle, engine, oeng, dmf, fwd_kernel):
    """dmf_forward_first_hits_device over P poses in one launch == the oracle per pose (every
    batched kernel, DMF_KNOB_FWD_KERNEL: 0 = the (tile block, pose) grid, 1 = per-XCD unit
    queues, 2 = per-wave lane refill k_forward_q; odd strides give partial 8x8 tiles)."""
    import ctypes as C
    from dmf_amd import _lib
    ov = Hh.oracle_volume(oracle, n=100)
    gv = Hh.gpu_volume(n=100)
    from dmf_amd import _lib as _l
    _l.set_knob(gv, "fwd_kernel", fwd_kernel)
    poses = Hh.all_poses()[:5].astype(np.float32)
    P, rd, cd = len(poses), 3, 2
    R, Cc = (H + rd - 1) // rd, (W + cd - 1) // cd
    L, h = gv._L, gv._h

    def dmalloc(nbytes):
        p = C.c_void_p()
        _lib.check(L.dmf_device_malloc(h, C.addressof(p), nbytes))
        return p.value
    dp, dk, ds = dmalloc(poses.nbytes), dmalloc(4 * P * R * Cc), dmalloc(4 * P * R * Cc)
    try:
        _lib.check(L.dmf_memcpy_h2d(h, dp, poses.ctypes.data, poses.nbytes))
        cam = _lib.make_camera(K, H, W)
        _lib.check(L.dmf_forward_first_hits_device(h, C.addressof(cam), dp, P, 10, 10, rd, cd, dk, ds, None))
        k = np.zeros(P * R * Cc, np.int32)
        _lib.check(L.dmf_memcpy_d2h(h, k.ctypes.data, dk, k.nbytes))
        k = k.reshape(P, -1)
        for p in range(P):
            ko, _ = oeng.forward_first_hits(ov, poses[p], 10, 10, rd, cd)
            assert np.array_equal(k[p], np.asarray(ko).reshape(-1)), p
        assert (k >= 0).any()
    finally:
        for p_ in (dp, dk, ds):
            L.dmf_device_free(h, p_)


@pytest.fixture(params=[57, 40])
def brick_variant(request):
    """A brick-pipeline fusion implementation (include/dmf_diag.h): 57 = DMF_FUSE_SLAB, the
    production kernel (slab walk on 20-B records, k_bk_fuse_s) at any grid; 40 =
    DMF_FUSE_CELL_WALK (per-cell walk on 24-B records, k_bk_fuse), an independent exact walk."""
    return request.param


def _brick_kernel(variant):
    return "dmf::k_bk_fuse_s<" if variant == 57 else "dmf::k_bk_fuse<"


@pytest.mark.parametrize("dims,nframes", [((128, 128, 128), 6),   # 4^3 bricks
                                          ((100, 100, 100), 3),   # partial edge bricks
                                          ((61, 50, 47), 3),      # odd dims, padded tiles
                                          ((32, 32, 32), 6)])     # one brick, ~30 parts: atomic flush
def test_fuse_brick_path(oracle, engine, dmf, brick_variant, dims, nframes):
    """Brick-owned fusion (k_bk_rays / k_bk_pairs / k_bk_fuse(_s), dmf_brick.hpp): the
    per-brick restart of the exact walk must give the oracle's counters bit for bit,
    for single-part bricks (plain adds) and multi-part bricks (device atomics)."""
    from dmf_amd import _lib
    poses, depth, _ = Hh.frames()
    poses = np.concatenate([poses, Hh.ref_style_poses()[:2]])[:nframes + 2]
    depth = np.concatenate([depth, depth[:2]])[:nframes + 2]
    ov = oracle.Volume()
    ov.setDimensions(*Hh.BOUNDS)
    ov.setVolumeSize(*dims)
    ov.constructVolume()
    ho, mo, so = oracle.fuse_depth(ov, K, depth, poses, dmin=200, dmax=1000)
    gv = dmf.VoxelVolume()
    gv.setDimensions(*Hh.BOUNDS)
    gv.setVolumeSize(*dims)
    gv.constructVolume()
    _lib.set_variant(gv, brick_variant)
    prm = dmf.FuseParams(dmin_mm=200, dmax_mm=1000)
    for _ in range(2):  # repeatable (LDS counters, work queue)
        hg, mg, sg = engine.fuse_depth(gv, depth, poses, prm)
        assert _lib.kernel_name(gv).startswith(_brick_kernel(brick_variant))
        assert np.array_equal(so, sg)
        assert np.array_equal(ho, hg) and np.array_equal(mo, mg)


def test_fuse_lds_box_kernel(oracle, engine, dmf):
    """k_fuse_l<12, 1280> (DMF_FUSE_LDS_BOX; the path for grids under 256 or over 1024 cells
    per axis) stays bit-exact now that the brick pipeline is the default."""
    from dmf_amd import _lib
    _, depth, _ = Hh.frames()
    poses = np.concatenate([Hh.ref_style_poses()[:2], Hh.frames()[0][:2]])
    frames = np.concatenate([depth[:2], depth[2:4]])
    ov = Hh.oracle_volume(oracle, n=96, clouds=[])
    ho, mo, so = oracle.fuse_depth(ov, K, frames, poses)
    gv = Hh.gpu_volume(n=96, clouds=[])
    _lib.set_variant(gv, 31)
    assert _lib.kernel_name(gv) == "dmf::k_fuse_l<12, 1280>"
    hg, mg, sg = engine.fuse_depth(gv, frames, poses)
    assert _lib.kernel_name(gv) == "dmf::k_fuse_l<12, 1280>"
    assert np.array_equal(so, sg) and np.array_equal(ho, hg) and np.array_equal(mo, mg)


def test_fuse_variant_controls(dmf):
    """dmf_diag.h: the fusion implementation and the knobs are per volume (a second volume
    keeps the defaults); unknown variants and knobs are rejected."""
    import ctypes as C
    from dmf_amd import _lib
    L = _lib.load()
    a, b = Hh.gpu_volume(n=64, clouds=[]), Hh.gpu_volume(n=64, clouds=[])
    _lib.set_variant(a, 40)
    _lib.set_knob(a, "pair_cap", 12345)
    va, vb, kb = C.c_int32(), C.c_int32(), C.c_int64()
    _lib.check(L.dmf_fuse_get_variant(a._h, C.addressof(va)))
    _lib.check(L.dmf_fuse_get_variant(b._h, C.addressof(vb)))
    _lib.check(L.dmf_volume_get_knob(b._h, _lib.KNOBS["pair_cap"], C.addressof(kb)))
    assert (va.value, vb.value, kb.value) == (40, 0, 0)
    assert _lib.kernel_name(a) == "dmf::k_bk_fuse<16, 8, 8>" and _lib.kernel_name(b).startswith("dmf::k_bk_fuse_s<")
    assert L.dmf_fuse_set_variant(a._h, 53) == _lib.DMF_ERR_INVALID
    assert L.dmf_volume_set_knob(a._h, 99, 1) == _lib.DMF_ERR_INVALID


def test_fuse_brick_vs_lds_box_full_size(dmf):
    """Size-independent check at the bench's grid (512^3, 8 frames of 640x480): the brick
    pipeline (default), k_fuse_l<12, 1280> (31) and the per-cell brick walk (40) are
    independent exact implementations of the same DDA spec and must agree counter for
    counter; every update is either a hit or a miss, and there is one hit per ray ending
    inside the grid."""
    import ctypes as C
    from dmf_amd import _lib, scene
    L = _lib.load()
    P = 8
    poses = np.ascontiguousarray(scene.fibonacci_poses(P, seed=1234), np.float32)
    depth = np.ascontiguousarray(scene.render_frames(scene.intrinsics(640, 480), 640, 480, poses), np.uint16)
    cam = _lib.make_camera(scene.intrinsics(640, 480), 480, 640)
    prm = _lib.default_fuse_params(dmin_mm=scene.DEPTH_MIN_MM, dmax_mm=scene.DEPTH_MAX_MM)
    vol = dmf.VoxelVolume()
    vol.setDimensions(*Hh.BOUNDS)
    vol.setVolumeSize(512, 512, 512)
    vol.constructVolume()
    h = vol._h
    nct = C.c_int64()
    _lib.check(L.dmf_fuse_counter_cells(h, C.addressof(nct)))
    nt = nct.value

    def dmalloc(nbytes):
        p = C.c_void_p()
        _lib.check(L.dmf_device_malloc(h, C.addressof(p), nbytes))
        return p.value
    dd, dp, dc, ds = dmalloc(depth.nbytes), dmalloc(poses.nbytes), dmalloc(8 * nt), dmalloc(64)
    _lib.check(L.dmf_memcpy_h2d(h, dd, depth.ctypes.data, depth.nbytes))
    _lib.check(L.dmf_memcpy_h2d(h, dp, poses.ctypes.data, poses.nbytes))
    out = {}
    try:
        for variant in (0, 31, 40):
            _lib.set_variant(vol, variant)
            _lib.check(L.dmf_memset_device(h, dc, 0, 8 * nt))
            _lib.check(L.dmf_memset_device(h, ds, 0, 64))
            _lib.check(L.dmf_fuse_depth_device(h, C.addressof(cam), dd, dp, P, C.addressof(prm), dc, dc + 4 * nt, ds))
            cnt = np.empty(2 * nt, np.int32)
            st = np.empty(8, np.uint64)
            _lib.check(L.dmf_memcpy_d2h(h, cnt.ctypes.data, dc, cnt.nbytes))
            _lib.check(L.dmf_memcpy_d2h(h, st.ctypes.data, ds, st.nbytes))
            out[variant] = (cnt, st)
    finally:
        for ptr_ in (dd, dp, dc, ds):
            L.dmf_device_free(h, ptr_)
    (c0, s0), (c1, s1), (c2, s2) = out[0], out[31], out[40]
    assert np.array_equal(s0[:4], s1[:4]) and np.array_equal(s0[:4], s2[:4]) and s0[3] == 0 and s0[0] > 10 ** 8
    assert np.array_equal(c0, c1) and np.array_equal(c0, c2)
    assert int(c0.astype(np.int64).sum()) == int(s0[0])  # hits + misses == cell updates
    assert int(c0[:nt].astype(np.int64).sum()) == int(s0[2])  # one hit per ray ending inside


@pytest.mark.parametrize("n,slots", [(256, 2048), (256, 16), (96, 64)])
def test_fuse_pass_a_hashed_histogram(oracle, dmf, n, slots):
    """Pass A's hashed histogram (the default above 8192 bricks, forced here with
    DMF_KNOB_A_HASH = slots words): 2048 words hold every workgroup's bricks; 16 / 64 words
    overflow in most workgroups, which k_bk_rays_recover then redoes with the direct table
    (the overflowed workgroups' first run writes ray records only).  Counters and statistics
    equal the oracle's either way."""
    from dmf_amd import _lib
    poses, depth, _ = Hh.frames()
    poses, depth = poses[:4], depth[:4]
    ov = Hh.oracle_volume(oracle, n=n, clouds=[])
    ho, mo, so = oracle.fuse_depth(ov, K, depth, poses, dmin=200, dmax=1000)
    gv = Hh.gpu_volume(n=n, clouds=[])
    _lib.set_variant(gv, 57)
    _lib.set_knob(gv, "a_hash", slots)
    eng = dmf.RayTracingEngine(dmf.Camera(K, H, W))
    hg, mg, sg = eng.fuse_depth(gv, depth, poses, dmf.FuseParams(dmin_mm=200, dmax_mm=1000))
    assert np.array_equal(so, sg), (so, sg)
    assert np.array_equal(ho, hg) and np.array_equal(mo, mg)


@pytest.mark.parametrize("mode", ["poses2", "paircap"])
def test_fuse_brick_multi_batch(oracle, engine, dmf, mode):
    """The brick pipeline (57 = the production slab walk on 20-B records, 40 = per-cell walk)
    cut into several pose batches accumulates the same counters as the oracle.  poses2: at
    most 2 poses per batch (DMF_KNOB_BATCH_POSES) over 5 frames; paircap: a pair capacity of
    1.6 x the largest frame's pairs (DMF_KNOB_PAIR_CAP), so the DEVICE cuts the batches by the
    pairs each frame really makes (k_bk_batches) and the host's geometric-bound launches past
    the device's batch count exit at once."""
    poses, depth, _ = Hh.frames()
    poses, depth = poses[:5], depth[:5]
    ov = Hh.oracle_volume(oracle, n=80, clouds=[])
    ho, mo, so = oracle.fuse_depth(ov, K, depth, poses, dmin=200, dmax=1000)
    gv = Hh.gpu_volume(n=80, clouds=[])
    from dmf_amd import _lib
    L = _lib.load()
    prm = dmf.FuseParams(dmin_mm=200, dmax_mm=1000)
    _lib.set_variant(gv, 57)  # the brick pipeline at this small grid
    if mode == "poses2":
        _lib.set_knob(gv, "batch_poses", 2)
        expect = 3
    else:  # pairs per frame from single-frame device calls (stats[4] = pairs)
        import ctypes as C
        import torch
        dev = torch.device("cuda", 0)
        gv.set_stream(torch.cuda.current_stream(dev).cuda_stream)
        nct = C.c_int64()
        _lib.check(L.dmf_fuse_counter_cells(gv._h, C.addressof(nct)))
        d_depth = torch.from_numpy(np.ascontiguousarray(depth).view(np.int16)).to(dev)
        d_poses = torch.from_numpy(np.ascontiguousarray(poses, np.float32)).to(dev)
        cam = _lib.make_camera(K, 480, 640)
        cnt = torch.zeros(2 * nct.value, dtype=torch.int32, device=dev)
        per = []
        for i in range(5):
            st = torch.zeros(8, dtype=torch.int64, device=dev)
            _lib.check(L.dmf_fuse_depth_device(gv._h, C.addressof(cam), d_depth[i].data_ptr(), d_poses[i].data_ptr(),
                                               1, C.addressof(prm), cnt.data_ptr(), cnt.data_ptr() + 4 * nct.value,
                                               st.data_ptr()))
            torch.cuda.synchronize(dev)
            per.append(int(st[4].item()))
        cap = int(1.6 * max(per))
        _lib.set_knob(gv, "pair_cap", cap)
        expect, acc = 0, None  # the greedy cut, restated
        for c in per:
            if acc is None or acc + c > cap:
                expect, acc = expect + 1, 0
            acc += c
        assert expect >= 3
    for variant, name in ((57, "dmf::k_bk_fuse_s<16, 32, 8>"), (40, "dmf::k_bk_fuse<16, 8, 8>")):
        _lib.set_variant(gv, variant)
        hg, mg, sg = engine.fuse_depth(gv, depth, poses, prm)
        assert _lib.kernel_name(gv) == name
        assert _lib.fuse_batches_used(gv) == expect
        assert np.array_equal(so, sg) and np.array_equal(ho, hg) and np.array_equal(mo, mg)


def _edge_fusion_cases():
    """Fusion inputs at the edges of the path: a ragged frame (61x37: packets hang over the
    right and bottom edges), exactly axis-aligned cameras (integer principal point: one ray
    per frame runs along a grid axis, its row and column are planar, and a constant depth
    puts every end on one plane), depths at the [dmin, dmax) bounds, frames with no valid
    pixel, and a camera whose rays all miss the grid."""
    from dmf_amd import scene
    cases = []
    Kr = np.array([60.0, 0.0, 30.3, 0.0, 60.0, 18.7, 0.0, 0.0, 1.0], np.float32)
    pr = scene.fibonacci_poses(3, seed=11)
    dr = np.stack([scene.render(Kr, 61, 37, T)[0] for T in pr])
    cases.append(("ragged", Kr, 37, 61, pr, dr))
    Ka = np.array([50.0, 0.0, 32.0, 0.0, 50.0, 24.0, 0.0, 0.0, 1.0], np.float32)

    def pose(R, t):
        return np.concatenate([np.asarray(R, np.float32), np.asarray(t, np.float32)[:, None]], 1).reshape(12)
    axis = np.stack([pose(np.eye(3), [0.0, 0.0, -0.9]),                       # looks along +z
                     pose([[0, 0, 1], [1, 0, 0], [0, 1, 0]], [-0.9, 0.0, 0.0]),   # along +x
                     pose([[1, 0, 0], [0, 0, -1], [0, 1, 0]], [0.0, 0.9, 0.0])])  # along -y
    plane = np.full((3, 48, 64), 600, np.uint16)
    ramp = np.tile(np.linspace(150, 1100, 64).astype(np.uint16), (48, 1))[None].repeat(3, 0)
    near = axis.copy()
    near[:, [3, 7, 11]] *= np.float32(0.6 / 0.9)  # 0.1 m from the grid face
    bounds = np.full((3, 48, 64), 200, np.uint16)
    bounds[:, ::2, :] = 1000  # dmin is valid, dmax is not
    cases += [("axis_plane", Ka, 48, 64, axis, plane), ("axis_ramp", Ka, 48, 64, axis, ramp),
              ("depth_bounds", Ka, 48, 64, near, bounds),
              ("ends_before_grid", Ka, 48, 64, axis, bounds),
              ("no_valid_pixel", Ka, 48, 64, axis, np.zeros((3, 48, 64), np.uint16)),
              ("misses_grid", Ka, 48, 64, pose(np.eye(3), [0.0, 0.0, 0.9])[None], plane[:1])]
    # non-finite and far poses: a NaN rotation (finite origin, NaN endpoints: the clip keeps
    # t0 = 0, t1 = 1 and the NaN end cell converts to the low clamp, as the oracle's x86
    # int64 conversion gives it), NaN / inf translations, a translation of 1e20 (nothing
    # reaches the grid)
    bad = np.stack([axis[0], axis[1], axis[2], axis[0]]).copy()
    bad[0, 0] = np.nan
    bad[1, 3] = np.nan
    bad[2, 7] = np.inf
    bad[3, 11] = np.float32(-1e20)
    cases.append(("nonfinite_poses", Ka, 48, 64, bad, np.concatenate([plane, plane[:1]])))
    return cases


def _diagonal_pose(origin):
    """Camera at `origin` looking along +(1, 1, 1) (its z axis), row-major 3x4."""
    z = np.ones(3) / np.sqrt(3.0)
    x = np.cross([0.0, 0.0, 1.0], z)
    x /= np.linalg.norm(x)
    y = np.cross(z, x)
    R = np.stack([x, y, z], 1)  # columns: camera axes in the world
    return np.concatenate([R, np.asarray(origin, float)[:, None]], 1).astype(np.float32).reshape(12)


@pytest.mark.parametrize("n", [512, 1024])
def test_fuse_long_rays_walk_fallback(oracle, dmf, n):
    """Rays that cross more than bk::kPathSteps = 32 brick boundaries: pass A records only the
    first 32 crossing axes, so pass B walks such rays again (bk_replay's fallback).  A camera
    outside a grid corner looking along the diagonal, depth 1.7 m: every ray crosses most of
    the grid (46+ boundaries at 512^3, 90+ at 1024^3), some packets mix them with shorter
    ones (the image corners).  Counters and statistics equal the oracle's."""
    from dmf_amd import _lib
    Kc = np.array([40.0, 0.0, 31.5, 0.0, 40.0, 23.5, 0.0, 0.0, 1.0], np.float32)
    P = np.stack([_diagonal_pose([-0.62, -0.6, -0.61]), _diagonal_pose([-0.6, -0.63, -0.6])])
    D = np.full((2, 48, 64), 1700, np.uint16)
    D[:, :8, :] = 600  # shorter rays (fewer than 32 boundaries) in the same packets as long ones
    ov = Hh.oracle_volume(oracle, n=n, clouds=[])
    gv = Hh.gpu_volume(n=n, clouds=[])
    ho, mo, so = oracle.fuse_depth(ov, Kc, D, P, dmin=200, dmax=2000)
    eng = dmf.RayTracingEngine(dmf.Camera(Kc, 48, 64))
    hg, mg, sg = eng.fuse_depth(gv, D, P, dmf.FuseParams(dmin_mm=200, dmax_mm=2000))
    assert _lib.kernel_name(gv) == "dmf::k_bk_fuse_s<16, 32, 8>"
    # rays average over 0.9 n cells (the diagonal ones cross ~47 boundaries at 512^3, ~94 at
    # 1024^3; the image's edge rays leave the grid earlier, under 32)
    assert so[0] / so[1] > 0.9 * n, so
    assert np.array_equal(so, sg), (so, sg)
    assert np.array_equal(ho, hg) and np.array_equal(mo, mg)


@pytest.mark.parametrize("n,variant", [(256, 0), (96, 57), (96, 40), (96, 31)])
def test_fuse_edge_cases(oracle, dmf, n, variant):
    """Every edge case of _edge_fusion_cases through (256, 0) the DEFAULT dispatch at a grid
    that takes the production kernel (the slab-walk brick pipeline on 20-B records,
    k_bk_fuse_s: axis-aligned rays exercise the zero |dq| minor axes of pack20's beta state),
    (96, 57) the same kernel at a small grid (several rays per brick boundary), (96, 40) the
    per-cell brick walk and (96, 31) k_fuse_l: counters and statistics equal the oracle's (zero
    where nothing is valid or nothing reaches the grid)."""
    from dmf_amd import _lib
    for name, Kc, Hc, Wc, P, D in _edge_fusion_cases():
        ov = Hh.oracle_volume(oracle, n=n, clouds=[])
        gv = Hh.gpu_volume(n=n, clouds=[])
        _lib.set_variant(gv, variant)
        ho, mo, so = oracle.fuse_depth(ov, Kc, D, P, dmin=200, dmax=1000)
        eng = dmf.RayTracingEngine(dmf.Camera(Kc, Hc, Wc))
        hg, mg, sg = eng.fuse_depth(gv, D, P, dmf.FuseParams(dmin_mm=200, dmax_mm=1000))
        if variant in (0, 57) and so[0] > 0:
            assert _lib.kernel_name(gv) == "dmf::k_bk_fuse_s<16, 32, 8>", name
        assert np.array_equal(so, sg), (name, so, sg)
        assert np.array_equal(ho, hg) and np.array_equal(mo, mg), name
        if name in ("no_valid_pixel", "misses_grid", "ends_before_grid"):
            assert so[0] == 0 and not hg.any() and not mg.any(), name
        else:
            assert so[0] > 0, name
