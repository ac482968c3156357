#!/usr/bin/env python3
"""A/B driver for fusion experiments (run on the GPU box, optionally under rocprofv3
--kernel-trace): the bench workload (config 4 shard: 128 poses of 640x480 into 512^3, or
--grid / --poses / --image) through the library named by DMF_LIB (default: the product
build), serial calls then pipelined calls, HIP-event timing; prints one JSON line with ms
per call in each mode and the log-odds digest of one call (== tests/golden when the
library is exact)."""
import argparse
import ctypes as C
import hashlib
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "depth-map-fusion-utils_amd")]
import dmf_amd  # noqa: E402
from dmf_amd import _lib, scene  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--grid", type=int, default=512)
ap.add_argument("--poses", type=int, default=128)
ap.add_argument("--image", default="640x480")
ap.add_argument("--calls", type=int, default=30)
ap.add_argument("--modes", default="serial,pipelined")
ap.add_argument("--tag", default=os.environ.get("DMF_LIB", "product"))
ap.add_argument("--knob", action="append", default=[], help="name=value (dmf_diag.h knob), repeatable")
a = ap.parse_args()
W, H = (int(x) for x in a.image.split("x"))
dev = torch.device("cuda", 0)
K = scene.intrinsics(W, H)
cache = f"/tmp/exp_depth_{W}x{H}_{a.poses}.npy"
poses = np.ascontiguousarray(scene.fibonacci_poses(a.poses, seed=1234), np.float32)
if os.path.exists(cache):
    depth = np.load(cache)
else:
    print(f"[exp_fuse] rendering {a.poses} frames", file=sys.stderr, flush=True)
    depth = np.ascontiguousarray(scene.render_frames(K, W, H, poses), np.uint16)
    np.save(cache, depth)
L = _lib.load()
vol = dmf_amd.VoxelVolume(0)
main = torch.cuda.Stream(dev)
inp = torch.cuda.Stream(dev)
vol.set_stream(main.cuda_stream)
vol.setDimensions(-0.5, 0.5, -0.5, 0.5, -0.5, 0.5)
vol.setVolumeSize(a.grid, a.grid, a.grid)
vol.constructVolume()
for kv in a.knob:
    k, val = kv.split("=")
    _lib.set_knob(vol, k, int(val))
cam = _lib.make_camera(K, H, W)
prm = _lib.default_fuse_params(dmin_mm=scene.DEPTH_MIN_MM, dmax_mm=scene.DEPTH_MAX_MM)
nct = C.c_int64()
_lib.check(L.dmf_fuse_counter_cells(vol._h, C.addressof(nct)))
nt = nct.value
d_depth = torch.from_numpy(depth.view(np.int16)).to(dev)
d_poses = torch.from_numpy(poses).to(dev)
cnt = torch.zeros(2 * nt, dtype=torch.int32, device=dev)
st = torch.zeros(8, dtype=torch.int64, device=dev)
P = a.poses


def call():
    _lib.check(L.dmf_fuse_depth_device(vol._h, C.addressof(cam), d_depth.data_ptr(), d_poses.data_ptr(), P,
                                       C.addressof(prm), cnt.data_ptr(), cnt.data_ptr() + 4 * nt, st.data_ptr()))


out = {"tag": a.tag, "knobs": a.knob, "grid": a.grid, "poses": P, "image": a.image, "kernel": None}
torch.cuda.synchronize(dev)
for mode in a.modes.split(","):
    print(f"[exp_fuse {a.tag}] mode {mode}", file=sys.stderr, flush=True)
    _lib.check(L.dmf_fuse_set_input_stream(vol._h, inp.cuda_stream if mode == "pipelined" else None))
    _lib.check(L.dmf_fuse_reserve(vol._h, C.addressof(cam), P, 0))
    cnt.zero_()
    st.zero_()
    torch.cuda.synchronize(dev)
    with torch.cuda.stream(main):
        call()
    torch.cuda.synchronize(dev)
    # the digest of every mode (== tests/golden when exact)
    lo = torch.empty(a.grid ** 3, dtype=torch.int16, device=dev)
    _lib.check(L.dmf_fuse_finalize_device(vol._h, cnt.data_ptr(), cnt.data_ptr() + 4 * nt, C.addressof(prm),
                                          lo.data_ptr()))
    torch.cuda.synchronize(dev)
    out[mode + "_digest"] = out["digest"] = hashlib.sha256(lo.cpu().numpy().tobytes()).hexdigest()[:16]
    out["updates"] = int(st[0].item())
    out["pairs"] = int(st[4].item())
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for _ in range(3):
        call()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    e0.record(main)
    for _ in range(a.calls):
        call()
    e1.record(main)
    torch.cuda.synchronize(dev)
    out[mode + "_ms"] = e0.elapsed_time(e1) / a.calls
    out[mode + "_wall_ms"] = (time.perf_counter() - t0) * 1e3 / a.calls
out["kernel"] = _lib.kernel_name(vol)
_lib.check(L.dmf_fuse_set_input_stream(vol._h, None))
print(json.dumps(out), flush=True)
