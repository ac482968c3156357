#!/usr/bin/env python3
"""A/B experiment: do two fusion pipelines on two streams co-run faster than back to back?

Two volumes (separate scratch and counters), the headline workload (128 x 640x480 -> 512^3)
each.  serial: every call on one stream; concurrent: volume k on stream k.  Prints ms per
fusion call for both (diagnostic for DESIGN.md 5.10: pass A / B of one call beside phase F
of the other)."""
import ctypes as C
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "depth-map-fusion-utils_amd")]
import bench  # noqa: E402
import dmf_amd  # noqa: E402
from dmf_amd import _lib, scene  # noqa: E402


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 200
    grid, P = 512, 128
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    poses, depth = bench.make_inputs(0, 1, P)
    K = scene.intrinsics(640, 480)
    d_depth = torch.from_numpy(depth.view(np.int16)).to(dev)
    d_poses = torch.from_numpy(np.ascontiguousarray(poses, np.float32)).to(dev)
    cam = _lib.make_camera(K, 480, 640)
    prm = _lib.default_fuse_params(dmin_mm=scene.DEPTH_MIN_MM, dmax_mm=scene.DEPTH_MAX_MM)
    streams = [torch.cuda.Stream(dev), torch.cuda.Stream(dev)]
    vols, bufs = [], []
    for k in range(2):
        v = dmf_amd.VoxelVolume(0)
        v.set_stream(streams[k].cuda_stream)
        v.setDimensions(-0.5, 0.5, -0.5, 0.5, -0.5, 0.5)
        v.setVolumeSize(grid, grid, grid)
        v.constructVolume()
        npad = C.c_int64()
        _lib.check(v._L.dmf_fuse_counter_cells_padded(v._h, 1, C.addressof(npad)))
        _lib.check(v._L.dmf_fuse_reserve(v._h, C.addressof(cam), P, 0))
        vols.append(v)
        bufs.append((torch.zeros(2 * npad.value, dtype=torch.int32, device=dev), npad.value))
    torch.cuda.synchronize()
    stats = torch.zeros(20, dtype=torch.int64, device=dev)

    def call(k):
        v = vols[k]
        c, npad = bufs[k]
        _lib.check(v._L.dmf_fuse_depth_device(v._h, C.addressof(cam), d_depth.data_ptr(), d_poses.data_ptr(), P,
                                              C.addressof(prm), c.data_ptr(), c.data_ptr() + 4 * npad, None))

    def run(n, concurrent):
        for k in range(2):
            vols[k].set_stream(streams[k if concurrent else 0].cuda_stream)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(n):
            call(i & 1)
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / n * 1e3

    run(10, False)
    run(10, True)
    for rep in range(3):
        s = run(steps, False)
        c = run(steps, True)
        print(f"rep {rep}: serial {s:.3f} ms/call, two streams {c:.3f} ms/call ({s / c:.3f}x)", flush=True)
    # results identical either way (integer counters): compare one call per volume
    for k in range(2):
        bufs[k][0].zero_()
    vols[0].set_stream(streams[0].cuda_stream)
    vols[1].set_stream(streams[0].cuda_stream)
    call(0)
    torch.cuda.synchronize()
    ref = bufs[0][0].clone()
    bufs[0][0].zero_()
    vols[0].set_stream(streams[0].cuda_stream)
    vols[1].set_stream(streams[1].cuda_stream)
    call(0)
    call(1)
    torch.cuda.synchronize()
    print("identical:", bool(torch.equal(ref, bufs[0][0])) and bool(torch.equal(ref, bufs[1][0])), flush=True)


if __name__ == "__main__":
    main()
