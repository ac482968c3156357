#!/usr/bin/env python3
"""A/B of the batched forward first-hits march (DMF_KNOB_FWD_KERNEL 0 = (tile block, pose) grid,
1 = per-XCD unit queues; argv[1] = comma-separated list, alternated) on bench.py's secondary
workload, dense 640x480 lattice at (10, 10, 1, 1), 128 poses per launch; outputs compared.
(Setup as tools/exp_reverse.py.)  Former: A/B of reverseRayTraceFast kernels (DMF_KNOB_REVERSE_KERNEL 0 = spatial order, 3 =
occupied_cells_ order, 4 = per-XCD unit queues; argv[1] = comma-separated list, alternated) on bench.py's secondary workload: a 512^3 volume integrated from 16
back-projected 640x480 frames, 128 poses per launch.  Prints ms per launch for each and
checks the visibility / good masks are identical (with a DMF_EXP_STATS library also the work
queue's lane occupancy: busy lane-iterations / 64 x burst iterations)."""
import ctypes as C
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "depth-map-fusion-utils_amd")]
import dmf_amd  # noqa: E402
from dmf_amd import _lib, scene  # noqa: E402

W, H, P, NI = 640, 480, 128, 16
dev = torch.device("cuda", 0)
K = scene.intrinsics(W, H)
poses = np.ascontiguousarray(scene.fibonacci_poses(P, seed=1234), np.float32)
cache = f"/tmp/exp_depth_{W}x{H}_{P}.npy"
depth = np.load(cache) if os.path.exists(cache) else np.ascontiguousarray(scene.render_frames(K, W, H, poses), np.uint16)
L = _lib.load()
vol = dmf_amd.VoxelVolume(0)
s = torch.cuda.current_stream(dev)
vol.set_stream(s.cuda_stream)
vol.setDimensions(-0.5, 0.5, -0.5, 0.5, -0.5, 0.5)
vol.setVolumeSize(512, 512, 512)
vol.constructVolume()
cam = _lib.make_camera(K, H, W)
d_depth = torch.from_numpy(depth.view(np.int16)).to(dev)
d_poses = torch.from_numpy(poses).to(dev)
xyz = torch.empty((NI, H, W, 3), dtype=torch.float32, device=dev)
_lib.check(L.dmf_backproject_device(vol._h, C.addressof(cam), d_depth.data_ptr(), d_poses.data_ptr(), NI, xyz.data_ptr()))
valid = (d_depth[:NI].view(torch.int16) > 0).reshape(-1)
pts = xyz.reshape(-1, 3)[valid].contiguous()
nrm = np.concatenate([scene.render(K, W, H, poses[i])[1].reshape(-1, 3) for i in range(NI)])
d_nrm = torch.from_numpy(nrm).to(dev).reshape(-1, 3)[valid].contiguous()
vol.integrate_device(pts.data_ptr(), d_nrm.data_ptr(), pts.shape[0])
V = vol.info()["num_occupied"]
words = (V + 63) // 64
out = {"voxels": int(V), "poses": P}
KS = [int(x) for x in sys.argv[1].split(",")] if len(sys.argv) > 1 else [0, 1, 0, 1]
res = {}
kb = torch.empty(P * H * W, dtype=torch.int32, device=dev)
sb = torch.empty(P * H * W, dtype=torch.int32, device=dev)
fst = torch.zeros(4, dtype=torch.int64, device=dev)
for kf in KS:
    _lib.set_knob(vol, "fwd_kernel", kf)

    def run():
        _lib.check(L.dmf_forward_first_hits_device(vol._h, C.addressof(cam), d_poses.data_ptr(), P, 10, 10, 1, 1,
                                                   kb.data_ptr(), sb.data_ptr(), fst.data_ptr()))
    run()
    torch.cuda.synchronize(dev)
    fst.zero_()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(5):
        run()
    e1.record(s)
    torch.cuda.synchronize(dev)
    out.setdefault(f"ms_fwd{kf}", []).append(round(e0.elapsed_time(e1) / 5, 4))
    out[f"samples_fwd{kf}"] = int(fst[0].item()) // 5
    if int(fst[1].item()) > 0:  # DMF_EXP_STATS library: lane utilisation of the march
        out[f"lane_util_fwd{kf}"] = round(int(fst[0].item()) / int(fst[1].item()), 4)
    res[kf] = (kb.cpu().numpy().copy(), sb.cpu().numpy().copy())
k0 = KS[0]
out["outputs_equal"] = bool(all(np.array_equal(res[k0][0], r[0]) and np.array_equal(res[k0][1], r[1]) for r in res.values()))
# the committed oracle digests of every pixel's (k, slot) (tests/golden/march_digests.json)
try:
    import hashlib
    gold = json.load(open(os.path.join(ROOT, "tests", "golden", "march_digests.json")))["config4_shard_N1"]
    dg = lambda a: hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()[:16]  # noqa: E731
    out["digest_match"] = bool(dg(res[k0][0]) == gold["forward_k_digest"] and dg(res[k0][1]) == gold["forward_slot_digest"])
except (OSError, KeyError) as e:
    out["digest_error"] = str(e)
print(json.dumps(out), flush=True)
