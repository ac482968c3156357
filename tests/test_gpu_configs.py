"""GPU: the fusion path at the single-GPU BASELINE.json configurations.

Each config is checked two ways:
* bit-exact against the CPU oracle (oracle.cpp dda_ray, OpenMP rows) on a frame subset at
  the config's FULL grid and image size;
* at the config's full pose count, through size-independent properties: the default
  dispatch and an independent exact implementation (brick pipeline vs k_fuse_l) agree
  counter for counter; every cell update is a hit or a miss; there is one hit per ray
  that ends inside the grid; the multi-batch brick path (pose batches sized by its pair
  budget) equals a single batch.
Configs: 2 = 640x480, 256^3, 64 poses; 3 = 1280x720, 512^3, 256 poses; 4 = 640x480,
512^3, 1024 poses over 8 GPUs: its per-GPU shard of 128 poses (the bench workload) against
the oracle on ALL 128 frames, and the 1024-pose one-GPU anchor; 5 = 1280x720, 1024^3, 2048
poses over 8 GPUs: its per-GPU shard of 256 poses (several pose batches of the brick
pipeline).  The reference sequence being scaled is the per-frame integration of
tests/Raytracing.cpp:70-76 / Volume.hpp:199-228.
"""
import ctypes as C
import json
import os

import numpy as np
import pytest

import helpers as Hh

pytestmark = pytest.mark.gpu

# the oracle's digests of bench.py's workloads at full size (tests/golden/gen_fusion_digests.py)
GOLDEN = json.load(open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "fusion_digests.json")))


class Fusion:
    """Device-API fusion of resident frames on one volume (torch tensors)."""

    def __init__(self, grid, W, H, P, seed=1234, shard=None):
        """shard = (world, rank): the rank's block of a P*world-pose sphere (bench.py
        make_inputs, dmf_amd.dist.shard_range)."""
        import torch
        import dmf_amd
        from dmf_amd import _lib, scene
        from dmf_amd import dist as D
        self.torch, self._lib = torch, _lib
        self.L = _lib.load()
        self.dev = torch.device("cuda", 0)
        self.K = scene.intrinsics(W, H)
        if shard is None:
            poses = scene.fibonacci_poses(P, seed=seed)
        else:
            world, rank = shard
            a, b = D.shard_range(P * world, world, rank)
            poses = scene.fibonacci_poses(P * world, seed=seed)[a:b]
        self.poses = np.ascontiguousarray(poses, np.float32)
        self.depth = np.ascontiguousarray(scene.render_frames(self.K, W, H, self.poses), np.uint16)
        self.vol = dmf_amd.VoxelVolume()
        self.vol.setDimensions(*Hh.BOUNDS)
        self.vol.setVolumeSize(grid, grid, grid)
        self.vol.constructVolume()
        self.vol.set_stream(torch.cuda.current_stream(self.dev).cuda_stream)
        self.cam = _lib.make_camera(self.K, H, W)
        self.prm = _lib.default_fuse_params(dmin_mm=scene.DEPTH_MIN_MM, dmax_mm=scene.DEPTH_MAX_MM)
        nct = C.c_int64()
        _lib.check(self.L.dmf_fuse_counter_cells(self.vol._h, C.addressof(nct)))
        self.nt = nct.value
        self.d_depth = torch.from_numpy(self.depth.view(np.int16)).to(self.dev)
        self.d_poses = torch.from_numpy(self.poses).to(self.dev)
        self.grid = grid

    def run(self, variant=0, p0=0, p1=None, counters=None):
        """Fuse frames [p0, p1) with `variant`; returns (tiled [hits | misses] int32 on the
        device, stats[8] uint64, kernel name)."""
        torch, L, _lib = self.torch, self.L, self._lib
        p1 = self.poses.shape[0] if p1 is None else p1
        c = torch.zeros(2 * self.nt, dtype=torch.int32, device=self.dev) if counters is None else counters
        st = torch.zeros(8, dtype=torch.int64, device=self.dev)
        _lib.set_variant(self.vol, variant)
        _lib.check(L.dmf_fuse_depth_device(self.vol._h, C.addressof(self.cam), self.d_depth[p0].data_ptr(),
                                           self.d_poses[p0].data_ptr(), p1 - p0, C.addressof(self.prm),
                                           c.data_ptr(), c.data_ptr() + 4 * self.nt, st.data_ptr()))
        name = _lib.kernel_name(self.vol)
        torch.cuda.synchronize(self.dev)
        return c, st.cpu().numpy().astype(np.uint64), name

    def digest(self, c):
        """sha256[:16] of the finalized x-major int16 log-odds of tiled counters c (bench.py
        logodds_digest, tests/golden/gen_fusion_digests.py)."""
        import hashlib
        torch, L, _lib = self.torch, self.L, self._lib
        lo = torch.empty(self.grid ** 3, dtype=torch.int16, device=self.dev)
        _lib.check(L.dmf_fuse_finalize_device(self.vol._h, c.data_ptr(), c.data_ptr() + 4 * self.nt,
                                              C.addressof(self.prm), lo.data_ptr()))
        torch.cuda.synchronize(self.dev)
        return hashlib.sha256(lo.cpu().numpy().tobytes()).hexdigest()[:16]

    def linear(self, c):
        """Tiled device counters -> x-major host (hits, misses)."""
        torch, L, _lib = self.torch, self.L, self._lib
        lin = torch.empty(self.grid ** 3, dtype=torch.int32, device=self.dev)
        out = []
        for half in (0, 1):
            _lib.check(L.dmf_fuse_counters_to_linear_device(self.vol._h, c.data_ptr() + 4 * self.nt * half,
                                                            lin.data_ptr()))
            torch.cuda.synchronize(self.dev)
            out.append(lin.cpu().numpy())
        return out


def _oracle_subset(oracle, f, frames):
    ov = oracle.Volume()
    ov.setDimensions(*Hh.BOUNDS)
    ov.setVolumeSize(f.grid, f.grid, f.grid)
    ov.constructVolume()
    from dmf_amd import scene
    return oracle.fuse_depth(ov, f.K, f.depth[frames], f.poses[frames], dmin=scene.DEPTH_MIN_MM,
                             dmax=scene.DEPTH_MAX_MM, threads=16)


def _invariants(f, c, st):
    hits = c[: f.nt].to(dtype=f.torch.int64).sum().item()
    total = c.to(dtype=f.torch.int64).sum().item()
    assert st[3] == 0  # DDA guard
    assert total == int(st[0])  # every update is a hit or a miss
    assert hits == int(st[2])   # one hit per ray ending inside the grid
    assert int(st[1]) > 0 and int(st[0]) > int(st[1])


@pytest.mark.parametrize("cfg", ["config2", "config3", "config5-shard"])
def test_config_oracle_subset(oracle, cfg):
    """Frame subset at the config's full grid and image size: bit-exact vs the oracle."""
    grid, W, H, frames = {"config2": (256, 640, 480, [0, 21, 42, 63]),
                          "config3": (512, 1280, 720, [0, 128]),
                          "config5-shard": (1024, 1280, 720, [5])}[cfg]
    P = {"config2": 64, "config3": 256, "config5-shard": 32}[cfg]
    f = Fusion(grid, W, H, P)
    ho, mo, so = _oracle_subset(oracle, f, frames)
    c = f.torch.zeros(2 * f.nt, dtype=f.torch.int32, device=f.dev)
    for p in frames:  # the default dispatch of this grid, one frame per call
        c, st, _ = f.run(0, p, p + 1, counters=c)
    hg, mg = f.linear(c)
    assert np.array_equal(hg, ho) and np.array_equal(mg, mo)


@pytest.mark.parametrize("cfg", ["config2", "config3", "config5-shard"])
def test_config_full_poses(cfg):
    """All of the config's poses (per GPU): default dispatch == the other exact kernel,
    counter for counter, plus the counting invariants."""
    grid, W, H, P = {"config2": (256, 640, 480, 64), "config3": (512, 1280, 720, 256),
                     "config5-shard": (1024, 1280, 720, 32)}[cfg]
    f = Fusion(grid, W, H, P)
    c0, s0, k0 = f.run(0)
    _invariants(f, c0, s0)
    gkey = {"config2": "config2_N1", "config3": "config3_N1"}.get(cfg)
    if gkey:  # bench.py's workload at N = 1: the committed oracle digest of all its frames
        assert f.digest(c0) == GOLDEN[gkey]["logodds_digest"] and int(s0[0]) == GOLDEN[gkey]["updates"]
    # the other exact kernels: k_fuse_l (or the slab-walk brick pipeline when the default is
    # k_fuse_l) and the per-cell-walk brick pipeline (variant 40)
    for other in (31 if k0.startswith("dmf::k_bk_fuse") else 57, 40):
        c1, s1, k1 = f.run(other)
        assert k0 != k1
        assert np.array_equal(s0[:4], s1[:4])
        assert f.torch.equal(c0, c1)
        del c1
    # every config's grid (256-1024 cells per axis) takes the slab-walk brick pipeline;
    # config 3's 256 frames are split into pose batches on it
    assert k0.startswith("dmf::k_bk_fuse_s")


def test_config5_shard_bench_workload_golden():
    """Config 5's per-GPU shard size as bench.py runs it at N = 1 (1280x720, 1024^3, the 256
    poses of fibonacci_poses(256)): the default call -- the slab-walk brick pipeline with pass
    A's hashed histogram (32768 bricks) -- equals the committed oracle digest of all 256
    frames (tests/golden/gen_fusion_digests.py config5_shard_N1)."""
    f = Fusion(1024, 1280, 720, 256)
    c0, s0, k0 = f.run(0)
    _invariants(f, c0, s0)
    assert k0.startswith("dmf::k_bk_fuse_s")
    g = GOLDEN["config5_shard_N1"]
    assert f.digest(c0) == g["logodds_digest"] and int(s0[0]) == g["updates"]


def test_config3_batches_equal_single_batch():
    """Config 3's frames through the brick pipeline in batches of 7 poses (48 frames: 7
    batches) == the default (one batch: the device's cut by the real pair count)."""
    f = Fusion(512, 1280, 720, 48, seed=99)
    c0, s0, _ = f.run(57)
    assert f._lib.fuse_batches_used(f.vol) == 1
    f._lib.set_knob(f.vol, "batch_poses", 7)
    c1, s1, _ = f.run(57)
    assert f._lib.fuse_batches_used(f.vol) == 7
    f._lib.set_knob(f.vol, "batch_poses", 0)
    assert np.array_equal(s0[:4], s1[:4]) and f.torch.equal(c0, c1)


def test_anisotropic_grid_over_8192_bricks(oracle):
    """1024 x 1024 x 288 cells = 9216 bricks (> 8192: the 1024-lane A/B
    workgroups with a 36 KiB LDS histogram) and unequal bricks per axis (bk_index, the
    brick decode in k_bk_fuse): brick pipeline == k_fuse_l counter for counter, and == the
    oracle on one frame."""
    import torch
    import dmf_amd
    from dmf_amd import _lib, scene
    L = _lib.load()
    dev = torch.device("cuda", 0)
    K = scene.intrinsics(640, 480)
    poses = np.ascontiguousarray(scene.fibonacci_poses(4, seed=3), np.float32)
    depth = np.ascontiguousarray(scene.render_frames(K, 640, 480, poses), np.uint16)
    dims = (1024, 1024, 288)
    bounds = (-0.5, 0.5, -0.5, 0.5, -0.5, 0.5 * 288 / 1024 * 2 - 0.5)  # exact binary deltas
    vol = dmf_amd.VoxelVolume()
    vol.setDimensions(*bounds)
    vol.setVolumeSize(*dims)
    vol.constructVolume()
    assert tuple(vol.dims) == dims
    vol.set_stream(torch.cuda.current_stream(dev).cuda_stream)
    cam = _lib.make_camera(K, 480, 640)
    prm = _lib.default_fuse_params(dmin_mm=scene.DEPTH_MIN_MM, dmax_mm=scene.DEPTH_MAX_MM)
    nct = C.c_int64()
    _lib.check(L.dmf_fuse_counter_cells(vol._h, C.addressof(nct)))
    nt = nct.value
    d_depth = torch.from_numpy(depth.view(np.int16)).to(dev)
    d_poses = torch.from_numpy(poses).to(dev)
    out = {}
    for variant in (57, 40, 31):
        _lib.set_variant(vol, variant)
        c = torch.zeros(2 * nt, dtype=torch.int32, device=dev)
        st = torch.zeros(8, dtype=torch.int64, device=dev)
        _lib.check(L.dmf_fuse_depth_device(vol._h, C.addressof(cam), d_depth.data_ptr(), d_poses.data_ptr(), 4,
                                           C.addressof(prm), c.data_ptr(), c.data_ptr() + 4 * nt, st.data_ptr()))
        torch.cuda.synchronize(dev)
        out[variant] = (c, st.cpu().numpy(), _lib.kernel_name(vol))
    (c0, s0, k0), (c1, s1, k1), (c2, s2, k2) = out[57], out[31], out[40]
    assert k0.startswith("dmf::k_bk_fuse_s") and k1.startswith("dmf::k_fuse_l") and k2.startswith("dmf::k_bk_fuse<")
    assert s0[0] > 10 ** 8 and np.array_equal(s0[:4], s1[:4]) and torch.equal(c0, c1)
    assert np.array_equal(s0[:4], s2[:4]) and torch.equal(c0, c2)
    # one frame against the oracle
    ov = oracle.Volume()
    ov.setDimensions(*bounds)
    ov.setVolumeSize(*dims)
    ov.constructVolume()
    ho, mo, _ = oracle.fuse_depth(ov, K, depth[2:3], poses[2:3], dmin=scene.DEPTH_MIN_MM, dmax=scene.DEPTH_MAX_MM,
                                  threads=16)
    _lib.set_variant(vol, 57)
    c = torch.zeros(2 * nt, dtype=torch.int32, device=dev)
    _lib.check(L.dmf_fuse_depth_device(vol._h, C.addressof(cam), d_depth[2].data_ptr(), d_poses[2].data_ptr(), 1,
                                       C.addressof(prm), c.data_ptr(), c.data_ptr() + 4 * nt, None))
    lin = torch.empty(int(np.prod(dims)), dtype=torch.int32, device=dev)
    for half, exp in ((0, ho), (1, mo)):
        _lib.check(L.dmf_fuse_counters_to_linear_device(vol._h, c.data_ptr() + 4 * nt * half, lin.data_ptr()))
        torch.cuda.synchronize(dev)
        assert np.array_equal(lin.cpu().numpy(), exp)


def _plan(f, P):
    """dmf_fuse_plan of this fusion call: (brick pipeline?, max pose batches)."""
    from dmf_amd import _lib
    info = _lib.fuse_plan(f.vol, f.cam, P)
    return info["brick"], info["max_batches"]


def test_config4_shard_all_frames_oracle(oracle):
    """BASELINE config 4's per-GPU shard = the bench workload (640x480, 512^3, the 128 poses
    of bench.py at N = 1): ALL 128 frames through the default dispatch in one call, bit-exact
    against the oracle fusing the same 128 frames at the full grid (OpenMP rows), plus the
    counting invariants; the per-cell-walk brick pipeline (variant 40) and k_fuse_l
    (variant 31) give the same counters."""
    f = Fusion(512, 640, 480, 128)
    c0, s0, k0 = f.run(0)
    assert k0.startswith("dmf::k_bk_fuse_s")
    _invariants(f, c0, s0)
    assert _plan(f, 128) == (1, 1)
    assert f.digest(c0) == GOLDEN["config4_shard_N1"]["logodds_digest"]
    hg, mg = f.linear(c0)
    ho, mo, so = _oracle_subset(oracle, f, list(range(128)))
    assert np.array_equal(so, s0[:3].astype(np.int64))
    assert np.array_equal(hg, ho) and np.array_equal(mg, mo)
    del hg, mg, ho, mo
    for other in (31, 40):
        c1, s1, k1 = f.run(other)
        assert k1 != k0 and np.array_equal(s0[:4], s1[:4]) and f.torch.equal(c0, c1)
        del c1


def test_config4_anchor_1024_poses():
    """Config 4's 1024 poses on ONE GPU (the strong-scaling anchor): the default call
    (several pose batches when the pair budget caps them) == k_fuse_l on all 1024 == the
    8 per-GPU shards of bench.py at N = 8 accumulated into one counter set (the sum the
    RCCL merge forms), counter for counter."""
    from dmf_amd import dist as D
    f = Fusion(512, 640, 480, 1024)
    c0, s0, k0 = f.run(0)
    assert k0.startswith("dmf::k_bk_fuse_s")
    _invariants(f, c0, s0)
    # the geometric bound would need several batches; the device's cut by the real pairs, one
    assert _plan(f, 1024)[1] > 1 and f._lib.fuse_batches_used(f.vol) == 1
    # the 1024 global poses of bench.py at N = 8: the committed oracle digest
    assert f.digest(c0) == GOLDEN["config4_N8_anchor"]["logodds_digest"]
    assert int(s0[0]) == GOLDEN["config4_N8_anchor"]["updates"]
    c1, s1, k1 = f.run(31)
    assert k1.startswith("dmf::k_fuse_l") and np.array_equal(s0[:4], s1[:4]) and f.torch.equal(c0, c1)
    del c1
    acc = f.torch.zeros_like(c0)
    tot = np.zeros(4, np.uint64)
    for r in range(8):
        a, b = D.shard_range(1024, 8, r)
        acc, st, _ = f.run(0, a, b, counters=acc)
        tot += st[:4]
    assert np.array_equal(tot, s0[:4]) and f.torch.equal(acc, c0)


def test_config5_shard_256_poses(oracle):
    """BASELINE config 5's per-GPU shard at its real size: 256 of the 2048 poses (rank 0's
    block) of 1280x720 depth into 1024^3.  The default call runs the brick pipeline (the
    geometric bound would cut it into several pose batches; the device cuts it by the pairs
    it really makes); it equals k_fuse_l counter for counter, satisfies the counting
    invariants, and two of its frames fused alone equal the oracle at the full grid."""
    f = Fusion(1024, 1280, 720, 256, shard=(8, 0))
    brick, batches = _plan(f, 256)
    assert brick == 1 and batches >= 1
    c0, s0, k0 = f.run(0)
    assert k0.startswith("dmf::k_bk_fuse_s")
    _invariants(f, c0, s0)
    assert f._lib.fuse_batches_used(f.vol) >= 1
    c1, s1, k1 = f.run(31)
    assert k1.startswith("dmf::k_fuse_l") and np.array_equal(s0[:4], s1[:4]) and f.torch.equal(c0, c1)
    del c0, c1
    frames = [0, 255]
    ho, mo, so = _oracle_subset(oracle, f, frames)
    c = f.torch.zeros(2 * f.nt, dtype=f.torch.int32, device=f.dev)
    for p in frames:
        c, st, _ = f.run(0, p, p + 1, counters=c)
    hg, mg = f.linear(c)
    assert np.array_equal(hg, ho) and np.array_equal(mg, mo)
