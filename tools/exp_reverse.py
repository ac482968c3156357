#!/usr/bin/env python3
"""A/B of reverseRayTraceFast kernels (DMF_KNOB_REVERSE_KERNEL 0 = spatial order, 3 =
occupied_cells_ order, 4 = per-XCD unit queues; argv[1] = comma-separated list, alternated;
argv[2] = comma-separated brick distance caps, DMF_KNOB_BDIST_CAP, 0 = default) on bench.py's secondary workload: a 512^3 volume integrated from 16
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
res = {}
KS = [int(x) for x in sys.argv[1].split(",")] if len(sys.argv) > 1 else [3, 0, 3, 0]
CAPS = [int(x) for x in sys.argv[2].split(",")] if len(sys.argv) > 2 else [0]
for cap, kr in [(c, k) for c in CAPS for k in KS]:
    tag = f"{kr}" if CAPS == [0] else f"{kr}_cap{cap}"
    _lib.set_knob(vol, "bdist_cap", cap)
    _lib.set_knob(vol, "reverse_kernel", kr)
    vis = torch.zeros(P * words, dtype=torch.int64, device=dev)
    good = torch.zeros(P * words, dtype=torch.int64, device=dev)
    st = torch.zeros(16, dtype=torch.int64, device=dev)

    def run():
        _lib.check(L.dmf_reverse_visibility_device(vol._h, C.addressof(cam), d_poses.data_ptr(), P, 0, vis.data_ptr(),
                                                   good.data_ptr(), st.data_ptr()))
    torch.cuda.synchronize(dev)
    f0, f1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    f0.record(s)
    run()  # the first call after a cap change rebuilds the distance field
    f1.record(s)
    torch.cuda.synchronize(dev)
    out[f"first_ms_kernel{tag}"] = f0.elapsed_time(f1)
    st.zero_()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(5):
        run()
    e1.record(s)
    torch.cuda.synchronize(dev)
    out[f"ms_kernel{tag}"] = e0.elapsed_time(e1) / 5
    out[f"samples_kernel{tag}"] = int(st[0].item()) // 5
    sv = st.cpu().numpy()
    if sv[10] > 0:  # DMF_EXP_STATS build: burst iterations (per wave) and busy lane-iterations
        out[f"lane_busy_kernel{tag}"] = float(sv[11]) / (64.0 * float(sv[10]))
    res[tag] = (vis.cpu().numpy(), good.cpu().numpy())
k0 = next(iter(res))
out["masks_equal"] = bool(all(np.array_equal(res[k0][0], r[0]) and np.array_equal(res[k0][1], r[1]) for r in res.values()))
# the committed oracle digest of every pose's good mask (tests/golden/march_digests.json)
try:
    import hashlib
    gold = json.load(open(os.path.join(ROOT, "tests", "golden", "march_digests.json")))["config4_shard_N1"]
    out["good_digest_match"] = {t: hashlib.sha256(r[1].astype("<i8").tobytes()).hexdigest()[:16] for t, r in res.items()}
    out["good_digest_expected"] = gold.get("reverse_good_digest")
except (OSError, KeyError) as e:
    out["good_digest_error"] = str(e)
print(json.dumps(out), flush=True)
