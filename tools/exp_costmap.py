#!/usr/bin/env python3
"""Timing of the collision cost map (round 5: A/B of an experiment build's DMF_KNOB_COST_SKIP, 0 =
empty-space jumps between 64-depth groups, -1 = off; argv[1] = comma-separated list, alternated;
the knob is gone from the product) on bench.py's secondary workload: 1024 centres on a 0.45 m
sphere (scene.sphere_centres) in the 512^3 volume integrated from 16 back-projected 640x480
frames.  Prints ms per launch for each, whether the maps are identical, and the map's digest
against tests/golden/march_digests.json (costmap_digest)."""
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
Vc = 1024
cp = scene.sphere_centres(Vc)
d_cp = torch.from_numpy(cp).to(dev)
cmap = torch.empty((Vc, Vc), dtype=torch.int32, device=dev)
out = {"centres": Vc}
res = {}
KS = [int(x) for x in sys.argv[1].split(",")] if len(sys.argv) > 1 else [0, -1, 0, -1]
for k in KS:
    if "cost_skip" in _lib.KNOBS:
        _lib.set_knob(vol, "cost_skip", k)

    def run():
        _lib.check(L.dmf_collision_cost_map_device(vol._h, d_cp.data_ptr(), Vc, cmap.data_ptr()))
    run()
    torch.cuda.synchronize(dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(5):
        run()
    e1.record(s)
    torch.cuda.synchronize(dev)
    out.setdefault(f"ms_skip{k}", []).append(round(e0.elapsed_time(e1) / 5, 4))
    res[k] = cmap.cpu().numpy().copy()
k0 = KS[0]
out["maps_equal"] = bool(all(np.array_equal(res[k0], r) for r in res.values()))
out["collided"] = int((res[k0] == 0x7FFFFFFF).sum())
import hashlib
out["digest"] = {k: hashlib.sha256(np.ascontiguousarray(r).tobytes()).hexdigest()[:16] for k, r in res.items()}
try:
    out["digest_expected"] = json.load(open(os.path.join(ROOT, "tests", "golden", "march_digests.json")))["config4_shard_N1"]["costmap_digest"]
except (OSError, KeyError) as e:
    out["digest_error"] = str(e)
print(json.dumps(out), flush=True)
