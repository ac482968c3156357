"""One rank of tests/test_gpu_boundary.py::test_rccl_world2_merge (run as a subprocess):
fuse this rank's pose shard, merge with libdmf's RCCL merge over a world-2 communicator
made by libdmf itself, and (rank 0) compare the merged log-odds with one rank fusing every
pose.  argv: rank, unique-id file, result file."""
import ctypes as C
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(HERE, "..", "depth-map-fusion-utils_amd"))
sys.path.insert(0, os.path.join(HERE, ".."))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import dmf_amd  # noqa: E402
from dmf_amd import _lib  # noqa: E402
from dmf_amd import dist as D  # noqa: E402
import helpers as Hh  # noqa: E402


def main():
    rank, uid_path, out_path = int(sys.argv[1]), sys.argv[2], sys.argv[3]
    world, n = 2, 61  # odd: the last tile row of a rank's slab is partial
    torch.cuda.set_device(rank)
    dev = torch.device("cuda", rank)
    L = _lib.load()
    uid = (C.c_char * 128)()
    if rank == 0:
        _lib.check(L.dmf_comm_unique_id(C.addressof(uid)))
        with open(uid_path + ".tmp", "wb") as f:
            f.write(bytes(uid))
        os.replace(uid_path + ".tmp", uid_path)
    else:
        t0 = time.time()
        while not os.path.exists(uid_path):
            if time.time() - t0 > 60:
                raise RuntimeError("no unique id from rank 0")
            time.sleep(0.05)
        C.memmove(uid, open(uid_path, "rb").read(), 128)
    comm = C.c_void_p()
    _lib.check(L.dmf_comm_init_rank(C.addressof(comm), world, C.addressof(uid), rank, rank))
    poses, depth, _ = Hh.frames()
    P = poses.shape[0]
    a, b = D.shard_range(P, world, rank)
    cam = _lib.make_camera(Hh.K, 480, 640)
    prm = _lib.default_fuse_params(dmin_mm=200, dmax_mm=1000)

    def volume():
        v = dmf_amd.VoxelVolume(rank)
        v.setDimensions(*Hh.BOUNDS)
        v.setVolumeSize(n, n, n)
        v.constructVolume()
        v.set_stream(torch.cuda.current_stream(dev).cuda_stream)
        return v

    def fused(v, p, d, ranks):
        npad = C.c_int64()
        _lib.check(L.dmf_fuse_counter_cells_padded(v._h, ranks, C.addressof(npad)))
        c = torch.zeros(2 * npad.value, dtype=torch.int32, device=dev)
        dd = torch.from_numpy(np.ascontiguousarray(d, np.uint16).view(np.int16)).to(dev)
        dp = torch.from_numpy(np.ascontiguousarray(p, np.float32)).to(dev)
        _lib.check(L.dmf_fuse_depth_device(v._h, C.addressof(cam), dd.data_ptr(), dp.data_ptr(), p.shape[0],
                                           C.addressof(prm), c.data_ptr(), c.data_ptr() + 4 * npad.value, None))
        return c, npad.value

    try:
        vol = volume()
        c, _ = fused(vol, poses[a:b], depth[a:b], world)
        nlo = C.c_int64()
        _lib.check(L.dmf_fuse_logodds_cells_padded(vol._h, world, C.addressof(nlo)))
        lo = torch.full((nlo.value,), 12345, dtype=torch.int16, device=dev)
        _lib.check(L.dmf_fuse_merge_finalize_device(vol._h, c.data_ptr(), C.addressof(prm), lo.data_ptr(), comm, None))
        torch.cuda.synchronize(dev)
        msg = "OK"
        if rank == 0:
            one = volume()
            c1, np1 = fused(one, poses, depth, 1)
            ref = torch.empty(n ** 3, dtype=torch.int16, device=dev)
            _lib.check(L.dmf_fuse_finalize_device(one._h, c1.data_ptr(), c1.data_ptr() + 4 * np1, C.addressof(prm),
                                                  ref.data_ptr()))
            torch.cuda.synchronize(dev)
            nbad = int((lo[: n ** 3] != ref).sum().item())
            msg = "OK" if nbad == 0 else f"FAIL {nbad} cells differ"
        open(out_path, "w").write(msg)
    finally:
        _lib.check(L.dmf_comm_destroy(comm))


if __name__ == "__main__":
    main()
