"""GPU: the query marches at the size the bench times them (bench.py secondary_reverse).

reverseRayTraceFast (RayTracingEngine.hpp:136-226, the function tests/SetCover.cpp:218-240
calls per candidate pose), the forward march's first hits (:280-308 sampling, every pixel) and
the Planner::run_tsp collision cost map (tests/CameraPathGen.cpp:310-331) over the bench's
secondary workload: 16 frames of the 640x480 Fibonacci sphere back-projected on the GPU and
integrated with their analytic normals into [-0.5, 0.5]^3 at 512^3 (config 4's shard) and
256^3 (config 2), then all 128 / 64 poses.  Every output is compared with the CPU oracle's
digest of the same workload (tests/golden/gen_march_digests.py, march_digests.json); pose 0's
and one middle pose's good lists and first hits are compared with the oracle run live.
"""
import ctypes as C
import json
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

GOLDEN = json.load(open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "march_digests.json")))


def _digest(a):
    import hashlib
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()[:16]


@pytest.mark.parametrize("key", ["config4_shard_N1", "config2_N1"])
def test_marches_at_bench_size(oracle, key):
    import torch
    import dmf_amd
    from dmf_amd import _lib, scene
    g = GOLDEN[key]
    grid, P, n_int, Vc = g["grid"], g["poses"], g["integrated_frames"], g["costmap_centres"]
    W, H = (int(x) for x in g["image"].split("x"))
    K = scene.intrinsics(W, H)
    poses = np.ascontiguousarray(scene.fibonacci_poses(P, seed=g["seed"]), np.float32)
    depth = scene.render_frames(K, W, H, poses[:n_int])
    dev = torch.device("cuda", 0)
    L = _lib.load()
    vol = dmf_amd.VoxelVolume()
    vol.setDimensions(-0.5, 0.5, -0.5, 0.5, -0.5, 0.5)
    vol.setVolumeSize(grid, grid, grid)
    vol.constructVolume()
    vol.set_stream(torch.cuda.current_stream(dev).cuda_stream)
    cam = _lib.make_camera(K, H, W)
    d_depth = torch.from_numpy(depth.view(np.int16)).to(dev)
    d_poses = torch.from_numpy(poses).to(dev)
    # the bench's volume: GPU back-projection (bit-exact with Camera.hpp:24-45) + analytic normals
    xyz = torch.empty((n_int, H, W, 3), dtype=torch.float32, device=dev)
    _lib.check(L.dmf_backproject_device(vol._h, C.addressof(cam), d_depth.data_ptr(), d_poses.data_ptr(), n_int,
                                        xyz.data_ptr()))
    valid = torch.from_numpy((depth > 0).reshape(-1)).to(dev)
    pts = xyz.reshape(-1, 3)[valid].contiguous()
    nrm = np.concatenate([scene.render(K, W, H, poses[i])[1].reshape(-1, 3) for i in range(n_int)])
    d_nrm = torch.from_numpy(nrm).to(dev)[valid].contiguous()
    vol.integrate_device(pts.data_ptr(), d_nrm.data_ptr(), pts.shape[0])
    occ = np.asarray(vol.occupied_cells_, np.uint64)
    assert occ.size == g["occupied"] and _digest(occ) == g["occupied_digest"]
    V = occ.size
    words = (V + 63) // 64
    good = torch.zeros(P * words, dtype=torch.int64, device=dev)
    _lib.check(L.dmf_reverse_visibility_device(vol._h, C.addressof(cam), d_poses.data_ptr(), P, 0, None,
                                               good.data_ptr(), None))
    k = torch.empty(P * H * W, dtype=torch.int32, device=dev)
    s = torch.empty(P * H * W, dtype=torch.int32, device=dev)
    _lib.check(L.dmf_forward_first_hits_device(vol._h, C.addressof(cam), d_poses.data_ptr(), P, 10, 10, 1, 1,
                                               k.data_ptr(), s.data_ptr(), None))
    cp = scene.sphere_centres(Vc)
    d_cp = torch.from_numpy(cp).to(dev)
    cmap = torch.empty((Vc, Vc), dtype=torch.int32, device=dev)
    _lib.check(L.dmf_collision_cost_map_device(vol._h, d_cp.data_ptr(), Vc, cmap.data_ptr()))
    torch.cuda.synchronize(dev)
    masks = good.cpu().numpy().view(np.uint64).reshape(P, words)
    kh, sh, cm = k.cpu().numpy(), s.cpu().numpy(), cmap.cpu().numpy()
    # live oracle on two poses (its own volume from the same points: the occupied lists agree)
    ov = oracle.Volume()
    ov.setDimensions(-0.5, 0.5, -0.5, 0.5, -0.5, 0.5)
    ov.setVolumeSize(grid, grid, grid)
    ov.constructVolume()
    ov.integratePointCloud(pts.cpu().numpy(), d_nrm.cpu().numpy())
    assert np.array_equal(ov.occupied_cells_, occ)
    oeng = oracle.Engine(K, H, W)
    for p in (0, P // 2 + 1):
        _, lst = oeng.reverseRayTraceFast(ov, poses[p], False)
        bits = np.unpackbits(masks[p].view(np.uint8), bitorder="little")
        assert not bits[V:].any()  # no bit past the last slot
        assert np.array_equal(occ[np.nonzero(bits[:V])[0]], np.asarray(lst, np.uint64)), p
        ko, ho = oeng.forward_first_hits(ov, poses[p], 10, 10, 1, 1)
        kp = kh.reshape(P, H, W)[p]
        assert np.array_equal(kp, ko), p
        sp = sh.reshape(P, H, W)[p]
        assert np.array_equal(occ[sp[kp >= 0]], ho[ko >= 0]) and (sp[kp < 0] == -1).all(), p
    # every pose / pixel / pair against the oracle's digests
    assert _digest(masks) == g["reverse_good_digest"]
    assert int(sum(int(np.unpackbits(m.view(np.uint8)).sum()) for m in masks)) == g["reverse_good_total"]
    assert int((kh >= 0).sum()) == g["forward_hit_rays"]
    assert _digest(kh) == g["forward_k_digest"] and _digest(sh) == g["forward_slot_digest"]
    assert int((cm == 0x7FFFFFFF).sum()) == g["costmap_collided"] and _digest(cm) == g["costmap_digest"]
    vol.close()
