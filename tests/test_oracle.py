"""CPU: the oracle against the committed golden vectors, against an independent
pure-Python restatement (oracle/py_oracle.py), and structural properties of the
DDA fusion spec.  No GPU."""
import ctypes as C
import os

import numpy as np
import pytest

from oracle import py_oracle as PY

GOLD = os.path.join(os.path.dirname(__file__), "golden", "golden_v1.npz")


@pytest.fixture(scope="module")
def gold():
    return np.load(GOLD)  # allow_pickle=False (default): our own fixture, data only


@pytest.fixture(scope="module")
def gold_cloud(gold, oracle):
    import sys
    sys.path.insert(0, os.path.dirname(GOLD))
    import gen_golden as G
    K, poses, depth = gold["K"], gold["poses"], gold["depth"]
    nrm16 = np.zeros((len(poses),) + gold["normals16"].shape[1:], np.float16)
    nrm16[:2] = gold["normals16"]
    return G, K, poses, depth, nrm16


def test_golden_regression(gold, gold_cloud, oracle):
    G, K, poses, depth, nrm16 = gold_cloud
    out = G.compute(K, poses, depth, nrm16)
    for k, v in out.items():
        assert np.array_equal(np.asarray(v), gold[k]), k


def test_golden_fixture_nontrivial(gold):
    assert len(gold["occ64"]) > 1000 and gold["rrtf64_counts"].sum() > 1000
    assert gold["fuse64_stats"][0] > 1e6 and (gold["min64"] > 0).all()
    assert (gold["fwd64_k"] >= 0).any() and (gold["zbuf64"] >= 0).any()


def _rand_poses(n, seed):
    from dmf_amd import scene
    rng = np.random.default_rng(seed)
    P = scene.fibonacci_poses(n, seed=seed)
    pts = rng.uniform(-0.3, 0.3, (n, 3)).astype(np.float32)
    nn = rng.normal(size=(n, 3)).astype(np.float32)
    nn /= np.linalg.norm(nn, axis=1, keepdims=True)
    return np.concatenate([P, scene.reference_style_poses(pts, nn)])


def test_camera_math_py_vs_cpp(oracle):
    rng = np.random.default_rng(1)
    from dmf_amd import scene
    K = scene.K_640x480
    for T in _rand_poses(8, 3):
        for _ in range(50):
            r, c, d = int(rng.integers(0, 480)), int(rng.integers(0, 640)), int(rng.integers(1, 3000))
            p = PY.project_point(K, r, c, d)
            assert np.array_equal(np.array(p, np.float32), oracle.project_point(K, r, c, d))
            w = PY.transform(T, p)
            assert np.array_equal(np.array(w, np.float32), oracle.transform_point(T, *[float(x) for x in p]))
        assert np.array_equal(PY.inverse(T), oracle.inverse_pose(T))
        for _ in range(50):
            x, y, z = rng.uniform(-1, 1), rng.uniform(-1, 1), rng.uniform(-0.2, 1.5)
            assert PY.deproject(K, x, y, z) == oracle.deproject_point(K, x, y, z)


def test_degree_and_angle(oracle):
    for rad in (0.0, 1.0, 1.5707963, 1.5882, 1.58824, 3.14159, 1e12, float("nan")):
        v = (rad * 180) / 3.14159
        exp = int(v) if np.isfinite(v) and -2**31 <= v < 2**31 else -2**31
        assert oracle.degree(rad) == exp


def test_angle_threshold_exhaustive(oracle):
    """libdmf evaluates degree(acosf(d)) in [0,90] as dstar <= d <= 1 on the GPU: check
    every float of the transition window and the edges against glibc acosf."""
    from dmf_amd import _lib
    f = C.c_float()
    _lib.check(_lib.load().dmf_angle_threshold(C.addressof(f)))
    dstar = np.float32(f.value)
    lo, hi = np.float32(-0.0180), np.float32(-0.0170)
    a, b = lo.view(np.uint32), hi.view(np.uint32)  # negative: a > b
    ds = np.arange(b, a + 1, dtype=np.uint32).view(np.float32)
    L = oracle.lib()
    v = np.array([1, 0, 0], np.float32)
    n = np.zeros(3, np.float32)
    bad = 0
    for d in ds:
        n[0] = d
        bad += bool(L.orc_angle_ok(n, v)) != bool(dstar <= d <= np.float32(1.0))
    assert bad == 0
    for d in (np.float32(1.0), np.nextafter(np.float32(1.0), np.float32(2)), np.float32(-1.0), np.float32(0.0),
              np.float32(-0.5), np.float32(0.99999)):
        n[0] = d
        assert bool(L.orc_angle_ok(n, v)) == bool(dstar <= d <= np.float32(1.0)), d


def test_integrate_and_reverse_py_vs_cpp(oracle, gold):
    K, poses, depth = gold["K"], gold["poses"], gold["depth"]
    W, H = int(gold["W"]), int(gold["H"])
    xyz = oracle.backproject(K, depth[0], poses[0])
    m = depth[0] > 0
    nrm = gold["normals16"][0][m].astype(np.float32)
    pts = xyz[m][::7]
    nrm = nrm[::7]
    bounds = (-0.5, 0.5, -0.5, 0.5, -0.5, 0.5)
    for n in (24, 30):
        pv = PY.Vol(bounds, (n, n, n))
        pv.integrate(pts, nrm)
        ov = oracle.Volume()
        ov.setDimensions(*bounds)
        ov.setVolumeSize(n, n, n)
        ov.constructVolume()
        ov.integratePointCloud(pts, nrm)
        assert np.array_equal(np.array(pv.occupied(), np.uint64), ov.occupied_cells_)
        eng = oracle.Engine(K, H, W)
        for T in gold["all_poses"][:6]:
            f1, g1 = PY.reverse_ray_trace_fast(pv, K, H, W, T)
            f2, g2 = eng.reverseRayTraceFast(ov, T, False)
            assert f1 == f2 and np.array_equal(np.array(g1, np.uint64), g2)


def _fuse_py(K, H, W, depth, poses, bounds, n, dmin, dmax):
    v = PY.Vol(bounds, (n, n, n))
    hits = np.zeros(n ** 3, np.int32)
    misses = np.zeros(n ** 3, np.int32)
    lin = lambda c: (c[0] * n + c[1]) * n + c[2]
    upd = 0
    for p in range(len(poses)):
        T = poses[p]
        O = (np.float32(T[3]), np.float32(T[7]), np.float32(T[11]))
        for r in range(H):
            for c in range(W):
                d = int(depth[p, r, c])
                if not (dmin <= d < dmax):
                    continue
                E = PY.transform(T, PY.project_point(K, r, c, d))
                inside = v.valid_points(E) and v.valid_coords(v.get_voxel(E))
                missed, hit = PY.dda_cells(v, O, E, inside)
                for cell in missed:
                    misses[lin(cell)] += 1
                if hit is not None:
                    hits[lin(hit)] += 1
                upd += len(missed) + (hit is not None)
    return hits, misses, upd


def test_dda_fusion_py_vs_cpp(oracle):
    """Exact-rational DDA (py_oracle, Fractions) vs the integer-scaled DDA (oracle.cpp)."""
    from dmf_amd import scene
    K = scene.K_640x480.copy()
    K[[0, 2, 4, 5]] *= np.float32(0.0625)  # 40x30 image
    W, H = 40, 30
    poses = _rand_poses(3, 11)
    depth = scene.render_frames(K, W, H, poses, dmin=1, dmax=65535)
    bounds = (-0.5, 0.5, -0.5, 0.5, -0.5, 0.5)
    for n in (16, 23):
        hp, mp, up = _fuse_py(K, H, W, depth, poses, bounds, n, 1, 65535)
        ov = oracle.Volume()
        ov.setDimensions(*bounds)
        ov.setVolumeSize(n, n, n)
        ov.constructVolume()
        ho, mo, so = oracle.fuse_depth(ov, K, depth, poses, dmin=1, dmax=65535)
        assert so[0] == up
        assert np.array_equal(hp, ho) and np.array_equal(mp, mo)


def test_dda_path_properties(oracle):
    """Every ray's cell path is 6-connected, ends at the endpoint cell (getVoxel of the
    back-projected point), and hits equal the binned endpoints (integratePointCloud)."""
    from dmf_amd import scene
    rng = np.random.default_rng(5)
    v = PY.Vol((-0.5, 0.5, -0.5, 0.5, -0.5, 0.5), (37, 37, 37))
    for _ in range(300):
        O = rng.uniform(-0.9, 0.9, 3).astype(np.float32)
        E = rng.uniform(-0.6, 0.6, 3).astype(np.float32)
        inside = v.valid_points(E) and v.valid_coords(v.get_voxel(E))
        missed, hit = PY.dda_cells(v, O, E, inside)
        path = missed + ([hit] if hit is not None else [])
        for a, b in zip(path, path[1:]):
            assert sum(abs(a[i] - b[i]) for i in range(3)) == 1
        assert all(v.valid_coords(c) for c in path)
        if inside:
            assert hit == v.get_voxel(E)
    # hits of a fused frame == occupancy of the binned back-projected cloud
    K = scene.K_640x480.copy()
    K[[0, 2, 4, 5]] *= np.float32(0.125)
    W, H = 80, 60
    poses = scene.fibonacci_poses(2, seed=3)
    depth = scene.render_frames(K, W, H, poses)
    ov = oracle.Volume()
    ov.setDimensions(-0.5, 0.5, -0.5, 0.5, -0.5, 0.5)
    ov.setVolumeSize(40, 40, 40)
    ov.constructVolume()
    h, m, st = oracle.fuse_depth(ov, K, depth, poses, dmin=200, dmax=1000)
    for i in range(2):
        xyz = oracle.backproject(K, depth[i], poses[i])
        ov.integratePointCloud(xyz[depth[i] > 0], np.zeros_like(xyz[depth[i] > 0]))
    assert np.array_equal(h > 0, ov.occupancy_dense().reshape(-1) > 0)
    assert st[2] == h.sum() and st[0] == h.sum() + m.sum()


def test_fusion_is_additive_over_pose_shards(oracle):
    """Counts are associative: fusing shards and summing == fusing all (multi-GPU merge)."""
    from dmf_amd import scene
    K = scene.K_640x480.copy()
    K[[0, 2, 4, 5]] *= np.float32(0.125)
    poses = scene.fibonacci_poses(4, seed=9)
    depth = scene.render_frames(K, 80, 60, poses)
    def vol():
        v = oracle.Volume()
        v.setDimensions(-0.5, 0.5, -0.5, 0.5, -0.5, 0.5)
        v.setVolumeSize(32, 32, 32)
        v.constructVolume()
        return v
    h, m, _ = oracle.fuse_depth(vol(), K, depth, poses)
    h1, m1, _ = oracle.fuse_depth(vol(), K, depth[:2], poses[:2])
    h2, m2, _ = oracle.fuse_depth(vol(), K, depth[2:], poses[2:])
    assert np.array_equal(h, h1 + h2) and np.array_equal(m, m1 + m2)
    L = oracle.fuse_finalize(h, m)
    assert L.min() >= -2000 and L.max() <= 3511


def test_greedy_set_cover_oracle_vs_python(oracle):
    """oracle.cpp greedySetCover restatement vs a direct Python transcription of
    Algorithms.hpp:38-86 (sorted lists, strict max in increasing id order, stop < 5)."""
    rng = np.random.default_rng(3)

    def ref(sets, min_gain=5):
        covered, ids, out = set(), list(range(len(sets))), []
        while True:
            sel, best = -1, 0
            for x in ids:
                d = len(set(sets[x]) - covered)
                if d > best:
                    best, sel = d, x
            if sel == -1 or best < min_gain:
                return out
            covered |= set(sets[sel])
            out.append(sel)
            ids.remove(sel)

    for trial in range(20):
        n = int(rng.integers(1, 30))
        universe = int(rng.integers(10, 400))
        sets = [np.unique(rng.integers(0, universe, int(rng.integers(0, 80)))).astype(np.uint64) for _ in range(n)]
        for mg in (1, 5):
            assert list(oracle.greedy_set_cover(sets, mg)) == ref([list(map(int, s)) for s in sets], mg)


def test_fuse_mt_equals_single_thread(oracle):
    """The OpenMP CPU baseline variant gives the same integer counts."""
    from dmf_amd import scene
    K = scene.K_640x480.copy()
    K[[0, 2, 4, 5]] *= np.float32(0.25)
    poses = scene.fibonacci_poses(3, seed=4)
    depth = scene.render_frames(K, 160, 120, poses)

    def vol():
        v = oracle.Volume()
        v.setDimensions(-0.5, 0.5, -0.5, 0.5, -0.5, 0.5)
        v.setVolumeSize(48, 48, 48)
        v.constructVolume()
        return v
    h1, m1, s1 = oracle.fuse_depth(vol(), K, depth, poses, dmin=200, dmax=1000)
    h4, m4, s4 = oracle.fuse_depth(vol(), K, depth, poses, dmin=200, dmax=1000, threads=4)
    assert np.array_equal(h1, h4) and np.array_equal(m1, m4) and np.array_equal(s1, s4)


def test_golden_config1_regression(oracle):
    """The oracle reproduces golden_config1.npz (config 1: 640x480, reference K, one pose)."""
    import sys
    sys.path.insert(0, os.path.dirname(GOLD))
    import gen_golden_config1 as G1
    z = np.load(os.path.join(os.path.dirname(GOLD), "golden_config1.npz"))
    out = G1.compute(z["K"], z["pose"], z["depth"], z["normals_q"])
    for k, v in out.items():
        assert np.array_equal(np.asarray(v), z[k]), k
    assert len(z["occ"]) > 1000 and len(z["rrtf_good"]) > 1000 and z["fuse_stats"][0] > 1e6


def test_collision_cost_map_py_vs_cpp(oracle, gold):
    """run_tsp cost map (tests/CameraPathGen.cpp:310-331): C++ restatement vs the pure-Python
    one, on short segments (<= ~0.4 m, i.e. <= 400 march steps each) through a 24^3 grid."""
    K, depth, poses = gold["K"], gold["depth"], gold["poses"]
    xyz = oracle.backproject(K, depth[0], poses[0])
    m = depth[0] > 0
    pts = xyz[m][::13]
    nrm = gold["normals16"][0][m][::13].astype(np.float32)
    bounds = (-0.5, 0.5, -0.5, 0.5, -0.5, 0.5)
    pv = PY.Vol(bounds, (24, 24, 24))
    pv.integrate(pts, nrm)
    ov = oracle.Volume()
    ov.setDimensions(*bounds)
    ov.setVolumeSize(24, 24, 24)
    ov.constructVolume()
    ov.integratePointCloud(pts, nrm)
    rng = np.random.default_rng(3)
    centres = rng.uniform(-0.2, 0.2, (9, 3)).astype(np.float32)
    centres[8] = centres[0]
    P = np.tile(np.eye(3, 4, dtype=np.float32).reshape(1, 12), (9, 1))
    P[:, 3::4] = centres
    got = oracle.collision_cost_map(ov, P)
    exp = PY.collision_cost_map(pv, centres)
    assert np.array_equal(got, exp)
    coll = got == 2 ** 31 - 1
    assert coll.any() and not coll.all()
    assert got[0, 8] == 0 and np.all(np.diag(got) == 0)


def test_fusion_digest_fixture_reproduces():
    """tests/golden/fusion_digests.json (the oracle digests bench.py and the GPU suite check
    against) is reproducible: config 2's entry (256^3, 64 frames of 640x480) regenerated by
    the same script equals the committed one, and every bench workload (config 4 at N = 1, 2,
    4, 8) has an entry."""
    import json
    import os
    import sys
    here = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
    sys.path.insert(0, here)
    import gen_fusion_digests as G
    table = json.load(open(os.path.join(here, "fusion_digests.json")))
    for k in ("config4_shard_N1", "config4_N2", "config4_N4", "config4_N8_anchor", "config2_N1"):
        assert k in table and len(table[k]["logodds_digest"]) == 16
    got = G.oracle_digest(*G.WORKLOADS["config2_N1"], threads=os.cpu_count() or 1)
    assert got == table["config2_N1"]
