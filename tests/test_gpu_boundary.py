"""GPU: the C-ABI contract of the fusion path beyond parity.

* dmf_fuse_depth_device only enqueues work (include/dmf.h): after dmf_fuse_reserve a
  fusion call issued behind a long spin kernel returns while its stream is still busy
  (no host synchronisation, no allocation), and the counters equal the oracle's.
* The multi-GPU merge entry points (dmf_fuse_allreduce_device,
  dmf_fuse_merge_finalize_device, dmf_flags_allreduce) over an RCCL communicator made by
  libdmf itself (dmf_comm_init_rank) and over torch's ProcessGroupNCCL communicator, at
  world size 1 (one GPU per box): merged log-odds equal the plain finalize; the world-2
  partition and schedule are covered on CPU by tests/test_dist.py.
* The merge's slab arithmetic at rank > 0 (dmf_fuse_merge_plan + the merge's own finalize
  step dmf_fuse_finalize_slab_device) for G = 2, 3, 8 emulated ranks on one GPU.
"""
import ctypes as C
import os

import numpy as np
import pytest

import helpers as Hh
from helpers import K

pytestmark = pytest.mark.gpu


def _setup(n=96, P=4):
    import torch
    import dmf_amd
    from dmf_amd import _lib
    L = _lib.load()
    poses, depth, _ = Hh.frames()
    poses = np.ascontiguousarray(poses[:P], np.float32)
    depth = np.ascontiguousarray(depth[:P], np.uint16)
    vol = dmf_amd.VoxelVolume()
    vol.setDimensions(*Hh.BOUNDS)
    vol.setVolumeSize(n, n, n)
    vol.constructVolume()
    dev = torch.device("cuda", 0)
    d_depth = torch.from_numpy(depth.view(np.int16)).to(dev)
    d_poses = torch.from_numpy(poses).to(dev)
    cam = _lib.make_camera(K, 480, 640)
    prm = _lib.default_fuse_params(dmin_mm=200, dmax_mm=1000)
    return torch, L, _lib, vol, dev, d_depth, d_poses, cam, prm, poses, depth


def _oracle_counts(oracle, depth, poses, n):
    ov = Hh.oracle_volume(oracle, n=n, clouds=[])
    return oracle.fuse_depth(ov, K, depth, poses, dmin=200, dmax=1000)


@pytest.mark.parametrize("n,variant", [(96, 57), (256, 0), (96, 40), (96, 31)])
def test_fuse_device_never_blocks_the_host(oracle, n, variant):
    """dmf_fuse_depth_device only enqueues (include/dmf.h; brick pipeline and the LDS-box
    kernel): with its stream held busy by a ~1 s spin kernel, the call returns while the
    stream is still busy (a host synchronisation inside would wait for the spin), and the
    counters then equal the oracle's.  A second call needs no new allocation either
    (dmf_fuse_reserve sized everything)."""
    import time
    torch, L, _lib, vol, dev, d_depth, d_poses, cam, prm, poses, depth = _setup(n)
    P = poses.shape[0]
    nct = C.c_int64()
    _lib.check(L.dmf_fuse_counter_cells(vol._h, C.addressof(nct)))
    nt = nct.value
    counters = torch.zeros(2 * nt, dtype=torch.int32, device=dev)
    lin = torch.empty(n ** 3, dtype=torch.int32, device=dev)
    s = torch.cuda.current_stream(dev)
    vol.set_stream(s.cuda_stream)
    _lib.set_variant(vol, variant)
    _lib.check(L.dmf_fuse_reserve(vol._h, C.addressof(cam), P, 0))

    def fuse():
        _lib.check(L.dmf_fuse_depth_device(vol._h, C.addressof(cam), d_depth.data_ptr(), d_poses.data_ptr(), P,
                                           C.addressof(prm), counters.data_ptr(), counters.data_ptr() + 4 * nt,
                                           None))
    fuse()  # first call: module loads
    torch.cuda.synchronize(dev)
    counters.zero_()
    for _ in range(2):
        torch.cuda._sleep(2_000_000_000)  # ~1 s of spinning at 2.1-2.4 GHz on the stream
        t0 = time.perf_counter()
        fuse()
        dt = time.perf_counter() - t0
        busy = not s.query()
        torch.cuda.synchronize(dev)
        assert busy and dt < 0.3, (busy, dt)
    ho, mo, _ = _oracle_counts(oracle, depth, poses, n)
    for half, exp in ((0, ho), (1, mo)):
        _lib.check(L.dmf_fuse_counters_to_linear_device(vol._h, counters.data_ptr() + 4 * nt * half,
                                                        lin.data_ptr()))
        torch.cuda.synchronize(dev)
        assert np.array_equal(lin.cpu().numpy(), 2 * exp)


def _fused_counters(torch, L, _lib, vol, dev, d_depth, d_poses, cam, prm, P, npad):
    counters = torch.zeros(2 * npad, dtype=torch.int32, device=dev)
    _lib.check(L.dmf_fuse_depth_device(vol._h, C.addressof(cam), d_depth.data_ptr(), d_poses.data_ptr(), P,
                                       C.addressof(prm), counters.data_ptr(), counters.data_ptr() + 4 * npad, None))
    return counters


@pytest.mark.parametrize("n", [96, 61])
def test_merge_entry_points_dmf_comm_world1(n):
    """dmf_comm_init_rank (world 1) + the three merge entry points: all-reduce leaves the
    counters unchanged, merge-finalize gives the plain finalize, flags stay put."""
    torch, L, _lib, vol, dev, d_depth, d_poses, cam, prm, poses, depth = _setup(n)
    P = poses.shape[0]
    vol.set_stream(torch.cuda.current_stream(dev).cuda_stream)
    ver = C.c_int32()
    _lib.check(L.dmf_rccl_version(C.addressof(ver)))
    assert ver.value > 20000
    uid = (C.c_char * 128)()
    _lib.check(L.dmf_comm_unique_id(C.addressof(uid)))
    comm = C.c_void_p()
    _lib.check(L.dmf_comm_init_rank(C.addressof(comm), 1, C.addressof(uid), 0, 0))
    try:
        npad, nlo, nct = C.c_int64(), C.c_int64(), C.c_int64()
        _lib.check(L.dmf_fuse_counter_cells_padded(vol._h, 1, C.addressof(npad)))
        _lib.check(L.dmf_fuse_logodds_cells_padded(vol._h, 1, C.addressof(nlo)))
        _lib.check(L.dmf_fuse_counter_cells(vol._h, C.addressof(nct)))
        assert npad.value >= nct.value and nlo.value >= n ** 3
        c = _fused_counters(torch, L, _lib, vol, dev, d_depth, d_poses, cam, prm, P, npad.value)
        ref_c = c.clone()
        ref = torch.empty(n ** 3, dtype=torch.int16, device=dev)
        _lib.check(L.dmf_fuse_finalize_device(vol._h, c.data_ptr(), c.data_ptr() + 4 * npad.value, C.addressof(prm),
                                              ref.data_ptr()))
        _lib.check(L.dmf_fuse_allreduce_device(vol._h, c.data_ptr(), npad.value, comm, None))
        torch.cuda.synchronize(dev)
        assert torch.equal(c, ref_c)
        lo = torch.full((nlo.value,), 12345, dtype=torch.int16, device=dev)
        side = torch.cuda.Stream(dev)  # the merge on a communication stream of its own
        side.wait_stream(torch.cuda.current_stream(dev))
        _lib.check(L.dmf_fuse_merge_finalize_device(vol._h, c.data_ptr(), C.addressof(prm), lo.data_ptr(), comm,
                                                    side.cuda_stream))
        torch.cuda.synchronize(dev)
        assert torch.equal(lo[: n ** 3], ref)
        # no communicator = a single rank: the finalize alone, on the given stream (bench N=1)
        lo1 = torch.full((nlo.value,), 12345, dtype=torch.int16, device=dev)
        side.wait_stream(torch.cuda.current_stream(dev))
        _lib.check(L.dmf_fuse_merge_finalize_device(vol._h, ref_c.data_ptr(), C.addressof(prm), lo1.data_ptr(), None,
                                                    side.cuda_stream))
        torch.cuda.synchronize(dev)
        assert torch.equal(lo1[: n ** 3], ref)
        # flags: integrate a cloud, set view/good by a query, all-reduce(max) at world 1
        pts, nn = Hh.cloud()
        vol.integratePointCloud(pts, nn)
        from dmf_amd import RayTracingEngine, Camera
        RayTracingEngine(Camera(K)).reverseRayTraceFast(vol, poses[0], True)
        view0, good0 = vol.voxel_flags()
        _lib.check(L.dmf_flags_allreduce(vol._h, comm, None))
        view1, good1 = vol.voxel_flags()
        assert np.array_equal(view0, view1) and np.array_equal(good0, good1) and view0.any()
    finally:
        _lib.check(L.dmf_comm_destroy(comm))


def test_merge_over_torch_process_group_world1(tmp_path):
    """The bench's path: torch's ProcessGroupNCCL communicator pointer handed to libdmf
    (one librccl instance in the process), merge-finalize == plain finalize.  (A file
    store: a free-port probe can race RCCL's own bootstrap sockets.)"""
    torch, L, _lib, vol, dev, d_depth, d_poses, cam, prm, poses, depth = _setup(80)
    import torch.distributed as dist
    from dmf_amd import dist as D
    import bench
    P = poses.shape[0]
    dist.init_process_group("nccl", init_method=f"file://{tmp_path / 'pg_store'}", rank=0, world_size=1,
                            device_id=dev)
    try:
        dist.barrier()
        assert bench.one_rccl_mapped()
        comm = D.torch_comm_ptr(device=dev)
        vol.set_stream(torch.cuda.current_stream(dev).cuda_stream)
        npad, nlo = C.c_int64(), C.c_int64()
        _lib.check(L.dmf_fuse_counter_cells_padded(vol._h, 1, C.addressof(npad)))
        _lib.check(L.dmf_fuse_logodds_cells_padded(vol._h, 1, C.addressof(nlo)))
        c = _fused_counters(torch, L, _lib, vol, dev, d_depth, d_poses, cam, prm, P, npad.value)
        ref = torch.empty(80 ** 3, dtype=torch.int16, device=dev)
        _lib.check(L.dmf_fuse_finalize_device(vol._h, c.data_ptr(), c.data_ptr() + 4 * npad.value, C.addressof(prm),
                                              ref.data_ptr()))
        lo = torch.zeros(nlo.value, dtype=torch.int16, device=dev)
        D.merge_finalize_device(vol, c, C.addressof(prm), lo, comm)
        torch.cuda.synchronize(dev)
        assert torch.equal(lo[: 80 ** 3], ref)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("dims", [(61, 61, 61), (1024, 1024, 288)])
@pytest.mark.parametrize("G", [2, 3, 8])
def test_merge_slabs_emulated_ranks(dims, G):
    """The multi-GPU merge's slab arithmetic at rank > 0, executed on one GPU:
    G ranks' counter replicas (seeded random counts, padded for G ranks), the reduce-scatter
    emulated with a device sum placed at each rank's chunk_offset (dmf_fuse_merge_plan), every
    rank's slab finalized by libdmf (dmf_fuse_finalize_slab_device, the merge's own finalize
    step), the slabs assembled at their slab_offset as the all-gather would: the result equals
    the plain finalize of the summed counters, and no rank writes outside its slab."""
    import torch
    import dmf_amd
    from dmf_amd import _lib
    L = _lib.load()
    dev = torch.device("cuda", 0)
    vol = dmf_amd.VoxelVolume()
    vol.setDimensions(0.0, dims[0] / 1024, 0.0, dims[1] / 1024, 0.0, dims[2] / 1024)  # exact 2^-10 deltas
    vol.setVolumeSize(*dims)
    vol.constructVolume()
    assert tuple(vol.dims) == dims
    vol.set_stream(torch.cuda.current_stream(dev).cuda_stream)
    prm = _lib.default_fuse_params()
    whole = _lib.merge_plan(vol, G, -1)
    npad, nlo = whole["n_padded"], whole["logodds_padded"]
    assert whole == _lib.merge_plan_dims(dims, G, -1)

    def replica(r):  # rank r's counters before the merge (deterministic, regenerated on demand)
        g = torch.Generator(device=dev)
        g.manual_seed(1000 + r)
        return torch.randint(0, 12, (2 * npad,), dtype=torch.int32, device=dev, generator=g)
    total = torch.zeros(2 * npad, dtype=torch.int32, device=dev)
    for r in range(G):
        total += replica(r)
    ref = torch.empty(nlo, dtype=torch.int16, device=dev)
    _lib.check(L.dmf_fuse_finalize_device(vol._h, total.data_ptr(), total.data_ptr() + 4 * npad, C.addressof(prm),
                                          ref.data_ptr()))
    out = torch.full((nlo,), -7, dtype=torch.int16, device=dev)  # the gathered grid
    outb = out.view(torch.uint8)
    covered = 0
    for r in range(G):
        p = _lib.merge_plan(vol, G, r)
        assert p == _lib.merge_plan_dims(dims, G, r)
        buf = replica(r)
        a, n = p["chunk_offset"], p["chunk"]
        buf[a:a + n] = total[a:a + n]                        # hits: this rank's reduced chunk
        buf[npad + a:npad + a + n] = total[npad + a:npad + a + n]  # misses
        lo = torch.full((nlo,), 12345, dtype=torch.int16, device=dev)
        _lib.check(L.dmf_fuse_finalize_slab_device(vol._h, buf.data_ptr(), C.addressof(prm), lo.data_ptr(), G, r,
                                                   None))
        torch.cuda.synchronize(dev)
        lob = lo.view(torch.uint8)
        s0, sb = p["slab_offset"], p["slab_bytes"]
        outb[s0:s0 + sb] = lob[s0:s0 + sb]
        # nothing outside the rank's own slab was written
        assert bool((lo[: s0 // 2] == 12345).all()) and bool((lo[(s0 + sb) // 2:] == 12345).all())
        covered += sb
        del buf, lo
    assert covered == 2 * nlo
    ncell = dims[0] * dims[1] * dims[2]
    assert torch.equal(out[:ncell], ref[:ncell])


def test_rccl_world2_merge(tmp_path):
    """World-2 RCCL merge across two GPUs: two processes, each fusing its pose
    shard of an odd 61^3 grid and merging through dmf_fuse_merge_finalize_device over a
    libdmf communicator; rank 0's merged log-odds equal one rank fusing every pose.  Runs
    only where the box has two GPUs (the builder's boxes have one: the slab arithmetic of
    ranks > 0 is covered by test_merge_slabs_emulated_ranks)."""
    import subprocess
    import sys
    import torch
    if torch.cuda.device_count() < 2:
        pytest.skip("needs two GPUs")
    worker = os.path.join(os.path.dirname(os.path.abspath(__file__)), "rccl_world2_worker.py")
    uid = str(tmp_path / "uid")
    outs = [str(tmp_path / f"r{r}.txt") for r in range(2)]
    procs = [subprocess.Popen([sys.executable, worker, str(r), uid, outs[r]]) for r in range(2)]
    try:
        rcs = [p.wait(timeout=150) for p in procs]
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    assert rcs == [0, 0], rcs
    assert open(outs[0]).read() == "OK" and open(outs[1]).read() == "OK"
