"""GPU: pipelined fusion (dmf_fuse_set_input_stream).

With an input stream declared, each call's pose table and pass A run on the volume's
staging stream into one of two slots and overlap the previous call's passes B and F.  The
counters and statistics must equal the serial order's exactly, also when
* the inputs are rewritten on the input stream before every call (the call must have made
  the input stream wait for its pass A),
* a call spans several super-batches (DMF_BK_SUPER_POSES: the slots alternate inside the
  call, slot reuse waits for the super-batch two back),
* the device cuts a super-batch into several pose batches (DMF_BK_BATCH_POSES),
* pass B is staged too (DMF_BK_STAGE=2: per-slot pair records, batch j+1's pass B after
  batch j's phase F),
and at 128^3 the sum over the calls equals the oracle's counters.
"""
import ctypes as C

import numpy as np
import pytest

import helpers as Hh

pytestmark = pytest.mark.gpu


def _frames(P):
    from dmf_amd import scene
    poses = np.ascontiguousarray(scene.fibonacci_poses(P, seed=77), np.float32)
    depth = np.ascontiguousarray(scene.render_frames(scene.intrinsics(640, 480), 640, 480, poses), np.uint16)
    return poses, depth


def _run(n, poses, depth, per_call, pipelined, variant=0):
    import torch
    import dmf_amd
    from dmf_amd import _lib, scene
    L = _lib.load()
    dev = torch.device("cuda", 0)
    vol = dmf_amd.VoxelVolume()
    vol.setDimensions(*Hh.BOUNDS)
    vol.setVolumeSize(n, n, n)
    vol.constructVolume()
    main = torch.cuda.Stream(dev)
    inp = torch.cuda.Stream(dev)
    vol.set_stream(main.cuda_stream)
    cam = _lib.make_camera(scene.intrinsics(640, 480), 480, 640)
    prm = _lib.default_fuse_params(dmin_mm=scene.DEPTH_MIN_MM, dmax_mm=scene.DEPTH_MAX_MM)
    nct = C.c_int64()
    _lib.check(L.dmf_fuse_counter_cells(vol._h, C.addressof(nct)))
    nt = nct.value
    all_depth = torch.from_numpy(depth.view(np.int16)).to(dev)
    all_poses = torch.from_numpy(poses).to(dev)
    # one input buffer of per_call frames, rewritten on the input stream before every call
    d_depth = torch.empty_like(all_depth[:per_call])
    d_poses = torch.empty_like(all_poses[:per_call])
    counters = torch.zeros(2 * nt, dtype=torch.int32, device=dev)
    stats = torch.zeros(8, dtype=torch.int64, device=dev)
    torch.cuda.synchronize(dev)
    _lib.check(L.dmf_fuse_set_variant(variant))
    try:
        if pipelined:
            _lib.check(L.dmf_fuse_set_input_stream(vol._h, inp.cuda_stream))
        _lib.check(L.dmf_fuse_reserve(vol._h, C.addressof(cam), per_call, 0))
        for c0 in range(0, poses.shape[0], per_call):
            with torch.cuda.stream(inp if pipelined else main):
                d_depth.copy_(all_depth[c0:c0 + per_call])
                d_poses.copy_(all_poses[c0:c0 + per_call])
            _lib.check(L.dmf_fuse_depth_device(vol._h, C.addressof(cam), d_depth.data_ptr(), d_poses.data_ptr(),
                                               per_call, C.addressof(prm), counters.data_ptr(),
                                               counters.data_ptr() + 4 * nt, stats.data_ptr()))
        torch.cuda.synchronize(dev)
        lin = torch.empty(n ** 3, dtype=torch.int32, device=dev)
        out = []
        for half in range(2):
            _lib.check(L.dmf_fuse_counters_to_linear_device(vol._h, counters.data_ptr() + 4 * nt * half,
                                                            lin.data_ptr()))
            vol.synchronize()
            out.append(lin.cpu().numpy())
        return out[0], out[1], stats.cpu().numpy()
    finally:
        _lib.check(L.dmf_fuse_set_input_stream(vol._h, None))
        _lib.check(L.dmf_fuse_set_variant(0))


@pytest.mark.parametrize("stage", ["1", "2"])
@pytest.mark.parametrize("case", ["calls", "super2", "super1_batches"])
def test_pipelined_equals_serial_256(monkeypatch, case, stage):
    """256^3 (the default brick pipeline), 4 calls of 3 frames; stage 1 = pass A staged,
    2 = pass A, the batch layout and pass B staged (DMF_BK_STAGE)."""
    monkeypatch.setenv("DMF_BK_STAGE", stage)
    poses, depth = _frames(12)
    if case == "super2":
        monkeypatch.setenv("DMF_BK_SUPER_POSES", "2")  # 3 frames -> super-batches of 2 + 1
    elif case == "super1_batches":
        monkeypatch.setenv("DMF_BK_SUPER_POSES", "3")
        monkeypatch.setenv("DMF_BK_BATCH_POSES", "1")  # three device batches per super-batch
    hs, ms, ss = _run(256, poses, depth, 3, pipelined=False)
    hp, mp, sp = _run(256, poses, depth, 3, pipelined=True)
    assert ss[0] > 10 ** 7 and ss[3] == 0
    # stats[5] (parts) differs by design: serial calls cut the part queue's tail (k_bk_scan),
    # pipelined ones do not; stats[6] (flushed cells) depends on which pairs share a part, i.e.
    # on the order of pass B's slot atomics, and varies run to run in either mode
    assert np.array_equal(ss[:5], sp[:5])
    assert np.array_equal(hs, hp) and np.array_equal(ms, mp)


@pytest.mark.parametrize("stage", ["1", "2"])
def test_pipelined_oracle_128(oracle, monkeypatch, stage):
    """128^3 through the brick pipeline (variant 57), 3 calls of 2 frames, vs the oracle."""
    monkeypatch.setenv("DMF_BK_STAGE", stage)
    poses, depth = _frames(6)
    hp, mp, sp = _run(128, poses, depth, 2, pipelined=True, variant=57)
    ov = oracle.Volume()
    ov.setDimensions(*Hh.BOUNDS)
    ov.setVolumeSize(128, 128, 128)
    ov.constructVolume()
    from dmf_amd import scene
    ho, mo, so = oracle.fuse_depth(ov, scene.intrinsics(640, 480), depth, poses,
                                   dmin=scene.DEPTH_MIN_MM, dmax=scene.DEPTH_MAX_MM)
    assert np.array_equal(np.asarray(so)[:3], sp[:3])
    assert np.array_equal(ho, hp) and np.array_equal(mo, mp)
