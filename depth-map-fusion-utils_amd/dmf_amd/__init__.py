"""dmf_amd — Python mirror of the reference Camera / VoxelVolume / RayTracingEngine
API (include/Camera.hpp, include/Volume.hpp, include/RayTracingEngine.hpp of
REXJJ/depth-map-fusion-utils) over the MI355X C ABI in libdmf.so.

Same class and method names, argument meaning and defaults as the reference, so
code written against the reference reads the same:

    cam = Camera(K)                                  # Camera.hpp:23
    volume = VoxelVolume()
    volume.setDimensions(xmin, xmax, ymin, ymax, zmin, zmax)
    volume.setVolumeSize(nx, ny, nz); volume.constructVolume()
    volume.integratePointCloud(xyz, normals)         # Volume.hpp:199-228
    engine = RayTracingEngine(cam)
    found, good = engine.reverseRayTraceFast(volume, pose, True)   # :136-226

Batched extensions (reverseRayTraceFastBatch, fuse_depth, ...) expose the GPU's
pose-parallelism.  Every compute call runs on the GPU through libdmf.so; there
is no CPU fallback.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib
from ._lib import DmfError, check, load, ptr

__all__ = ["Camera", "VoxelVolume", "RayTracingEngine", "OccupancyGrid", "DmfError", "degree", "FuseParams"]


def degree(radian):
    """CommonUtilities.hpp:17 degree(): int((radian*180)/3.14159)."""
    v = (float(radian) * 180) / 3.14159
    return int(v) if -2147483648.0 <= v < 2147483648.0 else -2147483648


class Camera:
    """Camera.hpp:17-86.  Scalar helpers are the reference formulas on the host;
    the per-pixel hot path (back-projection of whole frames) runs on the GPU."""

    def __init__(self, K, height=480, width=640):
        self.K_ = np.asarray(K, np.float32).reshape(9).copy()
        self.height_ = int(height)
        self.width_ = int(width)
        self._c = _lib.make_camera(self.K_, self.height_, self.width_)

    def getHeight(self):
        return self.height_

    def getWidth(self):
        return self.width_

    def validPixel(self, r, c):
        return 0 <= r < self.height_ and 0 <= c < self.width_

    def projectPoint(self, r, c, depth_mm):
        """Camera.hpp:24-31 (double math, float result)."""
        fx, cx, fy, cy = (float(self.K_[i]) for i in (0, 2, 4, 5))
        z = depth_mm * 0.001
        x = z * (float(c) - cx) / fx
        y = z * (float(r) - cy) / fy
        return np.float32(x), np.float32(y), np.float32(z)

    getPoint = projectPoint

    def deProjectPoint(self, x, y, z):
        """Camera.hpp:32-38: int(round((x*fx)/z + cx)) in double (C round: half away from 0)."""
        fx, cx, fy, cy = (float(self.K_[i]) for i in (0, 2, 4, 5))

        def cround_int(v):
            if not np.isfinite(v):
                return -2147483648
            v = float(np.sign(v) * np.floor(abs(v) + 0.5))
            return int(v) if -2147483648.0 <= v < 2147483648.0 else -2147483648

        with np.errstate(all="ignore"):
            c = cround_int(np.float64(x) * fx / np.float64(z) + cx)
            r = cround_int(np.float64(y) * fy / np.float64(z) + cy)
        return r, c

    def transformPoints(self, x, y, z, transformation):
        """Camera.hpp:39-45 (Eigen float affine, sum order a0+(a1+a2))."""
        m = np.asarray(transformation, np.float32).reshape(12)
        p = np.array([x, y, z], np.float32)
        out = []
        for i in range(3):
            s = m[4 * i + 0] * p[0] + (m[4 * i + 1] * p[1] + m[4 * i + 2] * p[2])
            out.append(np.float32(m[4 * i + 3] + s))
        return tuple(out)

    def getPixel(self, x, y, z, transformation=None):
        if transformation is None:
            transformation = np.array([1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0], np.float32)
        x, y, z = self.transformPoints(x, y, z, transformation)
        return self.deProjectPoint(x, y, z)

    def getAreaCovered(self, depth_mm):
        x1, y1, _ = (float(v) for v in self.getPoint(0, 0, depth_mm))
        x2, y2, _ = (float(v) for v in self.getPoint(0, self.height_, depth_mm))
        x3, y3, _ = (float(v) for v in self.getPoint(self.width_, 0, depth_mm))
        d = lambda a, b, c, e: np.sqrt((a - c) ** 2 + (b - e) ** 2)
        return np.float32(d(x1, y1, x2, y2) * d(x1, y1, x3, y3))

    def getDistance(self, depth_mm):
        x1, y1, _ = (float(v) for v in self.getPoint(100, 100, depth_mm))
        x2, y2, _ = (float(v) for v in self.getPoint(101, 101, depth_mm))
        return np.float32(np.sqrt((x1 - x2) ** 2 + (y1 - y2) ** 2))


class VoxelVolume:
    """Volume.hpp:50-255 VoxelVolume, device-resident (flat occupancy bitmask,
    dense slot map, occupied_cells_ list, CSR per-voxel points/normals)."""

    def __init__(self, device=0):
        self._L = load()
        h = C.c_void_p()
        check(self._L.dmf_volume_create(C.addressof(h), int(device)))
        self._h = h
        self._fields = {}

    def close(self):
        if getattr(self, "_h", None):
            self._L.dmf_volume_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # -- setup (Volume.hpp:89-128)
    def setDimensions(self, xmin, xmax, ymin, ymax, zmin, zmax):
        check(self._L.dmf_volume_set_dimensions(self._h, xmin, xmax, ymin, ymax, zmin, zmax))

    def setResolution(self, xdelta, ydelta, zdelta):
        check(self._L.dmf_volume_set_resolution(self._h, xdelta, ydelta, zdelta))

    def setVolumeSize(self, xdim, ydim, zdim):
        check(self._L.dmf_volume_set_volume_size(self._h, int(xdim), int(ydim), int(zdim)))

    def constructVolume(self):
        check(self._L.dmf_volume_construct(self._h))
        return True

    def set_stream(self, stream_ptr):
        check(self._L.dmf_volume_set_stream(self._h, stream_ptr))

    def set_fuse_input_stream(self, stream_ptr):
        """Pipelined fusion (dmf_fuse_set_input_stream): the device inputs of later fusion
        calls are ordered on stream_ptr; None restores the serial order."""
        check(self._L.dmf_fuse_set_input_stream(self._h, stream_ptr))

    def synchronize(self):
        check(self._L.dmf_volume_synchronize(self._h))

    def info(self):
        i = _lib.dmf_volume_info()
        check(self._L.dmf_volume_get_info(self._h, C.addressof(i)))
        return {f: getattr(i, f) for f, _ in i._fields_}

    def __getattr__(self, name):
        # public fields of the reference: xmin_, xdelta_, xdim_, hsize_, voxel_size_ ...
        if name.endswith("_") and not name.startswith("_"):
            key = name[:-1]
            inf = self.info()
            if key in inf:
                return inf[key]
        raise AttributeError(name)

    @property
    def dims(self):
        i = self.info()
        return i["xdim"], i["ydim"], i["zdim"]

    # -- hashing helpers (Volume.hpp:135-170, 230-233): host formulas
    def getHashId(self, x, y, z):
        return ((int(x) << 40) ^ ((int(y) << 20) & 0xFFFFFFFFFFFFFFFF) ^ int(z)) & 0xFFFFFFFFFFFFFFFF

    def getVoxel(self, x, y, z):
        i = self.info()
        f = lambda v, lo, d: int(np.floor((np.float64(np.float32(v)) - lo) / d))
        return f(x, i["xmin"], i["xdelta"]), f(y, i["ymin"], i["ydelta"]), f(z, i["zmin"], i["zdelta"])

    def getHash(self, x, y, z):
        return self.getHashId(*self.getVoxel(x, y, z))

    @staticmethod
    def getVoxelCoords(h):
        h = int(h)
        return h >> 40, (h >> 20) & ((1 << 20) - 1), h & ((1 << 20) - 1)

    def validCoords(self, x, y, z):
        nx, ny, nz = self.dims
        return 0 <= x < nx and 0 <= y < ny and 0 <= z < nz

    def validPoints(self, x, y, z):
        i = self.info()
        x, y, z = (np.float64(np.float32(v)) for v in (x, y, z))
        return not (x >= i["xmax"] or y >= i["ymax"] or z >= i["zmax"] or x <= i["xmin"] or y <= i["ymin"]
                    or z <= i["zmin"])

    # -- fusion of a point cloud (Volume.hpp:172-228), on the GPU
    def integratePointCloud(self, cloud, normals=None):
        xyz = np.ascontiguousarray(cloud, np.float32).reshape(-1, 3)
        nrm = None
        if normals is not None:
            nrm = np.ascontiguousarray(normals, np.float32).reshape(-1, 3)
            if nrm.shape != xyz.shape:
                raise ValueError("normals must match the cloud")
        nb = C.c_int64(0)
        hz = C.c_int64(0)
        check(self._L.dmf_volume_integrate(self._h, ptr(xyz), ptr(nrm), xyz.shape[0], C.addressof(nb),
                                           C.addressof(hz)))
        return True

    def integrate_device(self, d_xyz, d_normals, n):
        check(self._L.dmf_volume_integrate_device(self._h, d_xyz, d_normals, int(n)))

    @property
    def occupied_cells_(self):
        n = C.c_int64(0)
        check(self._L.dmf_volume_occupied(self._h, None, 0, C.addressof(n)))
        out = np.zeros(max(n.value, 1), np.uint64)
        check(self._L.dmf_volume_occupied(self._h, ptr(out), out.size, C.addressof(n)))
        return out[:n.value]

    def voxel_flags(self):
        """(view int32, good uint8) per occupied voxel in occupied_cells_ order."""
        V = self.info()["num_occupied"]
        view = np.zeros(max(V, 1), np.int32)
        good = np.zeros(max(V, 1), np.uint8)
        check(self._L.dmf_volume_voxel_flags(self._h, ptr(view), ptr(good), view.size))
        return view[:V], good[:V]

    def reset_flags(self):
        check(self._L.dmf_volume_reset_flags(self._h))

    def voxel_counts(self):
        V = self.info()["num_occupied"]
        a = np.zeros(max(V, 1), np.int64)
        b = np.zeros(max(V, 1), np.int64)
        check(self._L.dmf_volume_voxel_counts(self._h, ptr(a), ptr(b), a.size))
        return a[:V], b[:V]

    def voxel_points(self, hash_):
        n = C.c_int64(0)
        check(self._L.dmf_volume_voxel_points(self._h, int(hash_), None, None, 0, C.addressof(n)))
        if n.value < 0:
            return None, None
        p = np.zeros((max(n.value, 1), 3), np.float32)
        q = np.zeros((max(n.value, 1), 3), np.float32)
        check(self._L.dmf_volume_voxel_points(self._h, int(hash_), ptr(p), ptr(q), n.value, C.addressof(n)))
        return p[:n.value], q[:n.value]

    def occupancy_dense(self):
        nx, ny, nz = self.dims
        out = np.zeros(nx * ny * nz, np.uint8)
        check(self._L.dmf_volume_occupancy(self._h, ptr(out)))
        return out.reshape(nx, ny, nz)

    def getNeighborHashes(self, hash_, K=1):
        """Volume.hpp:235-255 (kept with the reference's `i==j==k==0` test)."""
        occ = self.occupancy_dense()
        x, y, z = self.getVoxelCoords(hash_)
        out = []
        for i in range(-K, K + 1):
            for j in range(-K, K + 1):
                for k in range(-K, K + 1):
                    if int(int(i == j) == k) == 0:
                        continue
                    a, b, c = x + i, y + j, z + k
                    if self.validCoords(a, b, c) and occ[a, b, c]:
                        out.append(self.getHashId(a, b, c))
        return out


def _pose(T):
    a = np.ascontiguousarray(T, np.float32).reshape(-1)
    if a.size == 16:
        a = np.ascontiguousarray(a.reshape(4, 4)[:3].reshape(12))
    if a.size != 12:
        raise ValueError("pose must be 3x4 (or 4x4) floats")
    return a


def _poses(T):
    """A stack of poses -> (P, 12) float32: each pose 3x4 or 4x4 (Eigen::Affine3f rows),
    a single pose, or already flattened rows of 12; anything else is rejected."""
    a = np.asarray(T, np.float32)
    if a.ndim == 2 and a.shape in ((3, 4), (4, 4)):
        a = a[None]
    if a.ndim == 3 and a.shape[1:] in ((3, 4), (4, 4)):
        return np.ascontiguousarray(a[:, :3, :].reshape(-1, 12))
    if a.ndim == 2 and a.shape[1] == 12:
        return np.ascontiguousarray(a)
    if a.ndim == 1 and a.size in (12, 16):
        return _pose(a)[None]
    raise ValueError(f"poses must be (P, 3, 4), (P, 4, 4) or (P, 12) floats, got shape {a.shape}")


class FuseParams:
    def __new__(cls, **kw):
        return _lib.default_fuse_params(**kw)


class RayTracingEngine:
    """RayTracingEngine.hpp:27-564 over the GPU.  Cheap to copy (holds only the camera)."""

    def __init__(self, cam):
        self.cam_ = cam

    def _c(self):
        return C.addressof(self.cam_._c)

    # reverseRayTraceFast  RayTracingEngine.hpp:136-226
    def reverseRayTraceFast(self, volume, transformation, viz, zdelta=1):
        found, lists = self.reverseRayTraceFastBatch(volume, _pose(transformation)[None], viz)
        return bool(found[0]), lists[0]

    def reverseRayTraceFastBatch(self, volume, poses, viz=False):
        return self._reverse(volume, poses, viz, volume._L.dmf_reverse_ray_trace_fast)

    # Set-cover consumer (Algorithms.hpp:38-86 greedySetCover over the
    # reverseRayTraceFast good sets, tests/SetCover.cpp:218-240): selected pose indices.
    def setCover(self, volume, poses, min_gain=5):
        poses = np.ascontiguousarray(np.asarray(poses, np.float32).reshape(-1, 12))
        P = poses.shape[0]
        sel = np.zeros(max(P, 1), np.int32)
        n = C.c_int32()
        check(volume._L.dmf_greedy_set_cover(volume._h, self._c(), ptr(poses), P, int(min_gain), ptr(sel),
                                             C.addressof(n)))
        return sel[:n.value]

    # reverseRayTrace  RayTracingEngine.hpp:45-134
    def reverseRayTrace(self, volume, transformation, viz, zdelta=1):
        found, lists = self._reverse(volume, _pose(transformation)[None], viz, volume._L.dmf_reverse_ray_trace)
        return bool(found[0]), lists[0]

    def _reverse(self, volume, poses, viz, fn):
        poses = np.ascontiguousarray(np.asarray(poses, np.float32).reshape(-1, 12))
        P = poses.shape[0]
        found = np.zeros(P, np.uint8)
        counts = np.zeros(P, np.int64)
        cap = max(int(volume.info()["num_occupied"]) * 2, 1024)
        while True:
            out = np.zeros(cap, np.uint64)
            st = fn(volume._h, self._c(), ptr(poses), P, int(bool(viz)), ptr(found), ptr(counts), ptr(out), cap)
            if st == _lib.DMF_ERR_CAPACITY:
                cap = int(counts.sum())
                continue
            check(st)
            break
        offs = np.concatenate([[0], np.cumsum(counts)])
        return found.astype(bool), [out[offs[i]:offs[i + 1]] for i in range(P)]

    # rayTrace  RayTracingEngine.hpp:268-309
    def rayTrace(self, volume, transformation, zdelta=10, sparse=True):
        check(volume._L.dmf_ray_trace(volume._h, self._c(), ptr(_pose(transformation)), int(zdelta), int(bool(sparse))))

    # rayTraceAndClassify  RayTracingEngine.hpp:311-375
    def rayTraceAndClassify(self, volume, transformation, zdelta=10, view=1, sparse=True):
        check(volume._L.dmf_ray_trace_and_classify(volume._h, self._c(), ptr(_pose(transformation)), int(zdelta),
                                                   int(view), int(bool(sparse))))

    # rayTraceAndGetMinimum  RayTracingEngine.hpp:229-264
    def rayTraceAndGetMinimum(self, volume, transformation, zdelta=1, sparse=True):
        m = C.c_int32(0)
        check(volume._L.dmf_ray_trace_and_get_minimum(volume._h, self._c(), ptr(_pose(transformation)), int(zdelta),
                                                      int(bool(sparse)), C.addressof(m)))
        return m.value

    def _fwd_list(self, fn, volume, transformation, zdelta, sparse):
        T = _pose(transformation)
        found = np.zeros(1, np.uint8)
        n = C.c_int64(0)
        cap = 1 << 16
        while True:
            out = np.zeros(cap, np.uint64)
            st = fn(volume._h, self._c(), ptr(T), int(zdelta), int(bool(sparse)), ptr(found), ptr(out), cap,
                    C.addressof(n))
            if st == _lib.DMF_ERR_CAPACITY:
                cap = n.value
                continue
            check(st)
            return bool(found[0]), out[:n.value]

    # rayTraceAndGetGoodPoints  RayTracingEngine.hpp:377-445
    def rayTraceAndGetGoodPoints(self, volume, transformation, zdelta=10, sparse=True):
        return self._fwd_list(volume._L.dmf_ray_trace_and_get_good_points, volume, transformation, zdelta, sparse)

    # rayTraceAndGetPoints  RayTracingEngine.hpp:447-494
    def rayTraceAndGetPoints(self, volume, transformation, zdelta=10, sparse=True):
        return self._fwd_list(volume._L.dmf_ray_trace_and_get_points, volume, transformation, zdelta, sparse)

    def forward_first_hits(self, volume, transformation, zstart, zdelta, rdelta, cdelta):
        H, W = self.cam_.height_, self.cam_.width_
        R, Cc = (H + rdelta - 1) // rdelta, (W + cdelta - 1) // cdelta
        k = np.zeros(R * Cc, np.int32)
        h = np.zeros(R * Cc, np.uint64)
        check(volume._L.dmf_forward_first_hits(volume._h, self._c(), ptr(_pose(transformation)), zstart, zdelta,
                                               rdelta, cdelta, ptr(k), ptr(h)))
        return k.reshape(R, Cc), h.reshape(R, Cc)

    # rayTraceVolume  RayTracingEngine.hpp:498-564
    def rayTraceVolume(self, volume, transformation):
        d = np.zeros(self.cam_.height_ * self.cam_.width_, np.int32)
        check(volume._L.dmf_ray_trace_volume(volume._h, self._c(), ptr(_pose(transformation)), ptr(d)))
        return d.reshape(self.cam_.height_, self.cam_.width_)

    # back-projection of whole frames (Camera.hpp:24-45), on the GPU
    def backproject(self, volume, depth, transformation):
        depth = np.ascontiguousarray(depth, np.uint16)
        out = np.zeros(depth.shape + (3,), np.float32)
        check(volume._L.dmf_backproject(volume._h, self._c(), ptr(depth), ptr(_pose(transformation)), ptr(out)))
        return out

    # 3D-DDA log-odds fusion
    def fuse_depth(self, volume, depth, poses, params=None, hits=None, misses=None):
        depth = np.ascontiguousarray(depth, np.uint16)
        if depth.ndim == 2:
            depth = depth[None]
        poses = _poses(poses)
        H, W = self.cam_.height_, self.cam_.width_
        if depth.shape != (poses.shape[0], H, W):
            raise ValueError(f"depth must be (P, H, W) = ({poses.shape[0]}, {H}, {W}) uint16, got {depth.shape}")
        n = int(np.prod(volume.dims))
        for name, a in (("hits", hits), ("misses", misses)):
            if a is not None and not (isinstance(a, np.ndarray) and a.dtype == np.int32 and a.size == n
                                      and a.flags.c_contiguous):
                raise ValueError(f"{name} must be a contiguous int32 array of {n} cells (accumulated in place)")
        hits = np.zeros(n, np.int32) if hits is None else hits
        misses = np.zeros(n, np.int32) if misses is None else misses
        stats = np.zeros(3, np.int64)
        params = params or _lib.default_fuse_params()
        check(volume._L.dmf_fuse_depth(volume._h, self._c(), ptr(depth), ptr(poses), poses.shape[0],
                                       C.addressof(params), ptr(hits), ptr(misses), ptr(stats)))
        return hits, misses, stats

    def fuse_finalize(self, volume, hits, misses, params=None):
        params = params or _lib.default_fuse_params()
        out = np.zeros(hits.size, np.int16)
        check(volume._L.dmf_fuse_finalize(volume._h, ptr(np.ascontiguousarray(hits, np.int32)),
                                          ptr(np.ascontiguousarray(misses, np.int32)), C.addressof(params), ptr(out)))
        return out


def will_collide(volume, a, b):
    """tests/CameraPathGen.cpp:128-156 willCollide, batched over segment pairs."""
    a = np.ascontiguousarray(a, np.float32).reshape(-1, 3)
    b = np.ascontiguousarray(b, np.float32).reshape(-1, 3)
    out = np.zeros(a.shape[0], np.uint8)
    check(volume._L.dmf_will_collide(volume._h, ptr(a), ptr(b), a.shape[0], ptr(out)))
    return out.astype(bool)


def collision_cost_map(volume, poses):
    """Planner::run_tsp cost map (tests/CameraPathGen.cpp:310-331): (V, V) int32 over the
    camera centres of `poses` (V x 3x4), INT_MAX where willCollide, else int(dist * 1000)."""
    poses = np.ascontiguousarray(poses, np.float32).reshape(-1, 12)
    V = poses.shape[0]
    out = np.zeros((V, V), np.int32)
    check(volume._L.dmf_collision_cost_map(volume._h, ptr(poses), V, ptr(out)))
    return out


class OccupancyGrid:
    """OccupancyGrid.hpp:50-318 on the GPU (dmf_ogrid_*): same setup sequence
    (setDimensions, setResolution, setK, construct), updateStates(cloud, normals) and the
    download calls.  updateStates gives the deterministic single-threaded result."""

    def __init__(self, device=0):
        self._L = load()
        h = C.c_void_p()
        check(self._L.dmf_ogrid_create(C.addressof(h), int(device)))
        self._h = h
        self._b = None
        self._r = None
        self.k_ = 0

    def close(self):
        if getattr(self, "_h", None):
            self._L.dmf_ogrid_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def setDimensions(self, xmin, xmax, ymin, ymax, zmin, zmax):
        self._b = np.array([xmin, xmax, ymin, ymax, zmin, zmax], np.float64)

    def setResolution(self, x, y, z):
        self._r = (float(np.float32(x)), float(np.float32(y)), float(np.float32(z)))

    def setK(self, k):
        self.k_ = int(k)

    def construct(self):
        check(self._L.dmf_ogrid_setup(self._h, ptr(self._b), *self._r, self.k_))
        return True

    @property
    def dims(self):
        d = np.zeros(3, np.int32)
        check(self._L.dmf_ogrid_get_dims(self._h, ptr(d)))
        return tuple(int(x) for x in d)

    def updateStates(self, cloud, normals):
        """cloud (n,3) xyz; normals (m,6) x y z nx ny nz (PointNormal)."""
        cloud = np.ascontiguousarray(cloud, np.float32).reshape(-1, 3)
        normals = np.ascontiguousarray(normals, np.float32).reshape(-1, 6)
        check(self._L.dmf_ogrid_update_states(self._h, ptr(cloud), cloud.shape[0], ptr(normals), normals.shape[0]))
        return True

    def state(self):
        n = int(np.prod(self.dims))
        nrm, cen = np.zeros(3 * n, np.float32), np.zeros(3 * n, np.float32)
        cnt, fl = np.zeros(n, np.int32), np.zeros(n, np.uint8)
        check(self._L.dmf_ogrid_state(self._h, ptr(nrm), ptr(cen), ptr(cnt), ptr(fl)))
        return nrm.reshape(-1, 3), cen.reshape(-1, 3), cnt, fl

    def _download(self, mode):
        n = C.c_int64()
        st = self._L.dmf_ogrid_download(self._h, mode, None, 0, C.addressof(n))
        if st not in (0, _lib.DMF_ERR_CAPACITY):
            check(st)
        out = np.zeros(6 * max(n.value, 1), np.float32)
        check(self._L.dmf_ogrid_download(self._h, mode, ptr(out), n.value, C.addressof(n)))
        return out[:6 * n.value].reshape(-1, 6)

    def downloadCloud(self):
        """(n, 6) centroid xyz + normal of occupied voxels, x-major (:166-193)."""
        return self._download(0)

    def downloadHQCloud(self):
        """as downloadCloud for voxels with count > 100 (:283-318)."""
        return self._download(1)

    def downloadReorganizedCloud(self, clean=False):
        """(n, 6) of the reorganized grid (:200-286): every occupied voxel (with clean,
        count >= 100) merges into the voxel holding its centroid, in the single-threaded
        x-major order; occupied reorganized voxels, x-major."""
        return self._download(3 if clean else 2)

    def set_state(self, normal, centroid, count, flags):
        """Write the dense voxels_ fields (normal, centroid (n, 3) float; count int32;
        flags occupied | normal_found << 1) — the reference's public state."""
        n = int(np.prod(self.dims))
        nrm = np.ascontiguousarray(normal, np.float32).reshape(3 * n)
        cen = np.ascontiguousarray(centroid, np.float32).reshape(3 * n)
        cnt = np.ascontiguousarray(count, np.int32).reshape(n)
        fl = np.ascontiguousarray(flags, np.uint8).reshape(n)
        check(self._L.dmf_ogrid_set_state(self._h, ptr(nrm), ptr(cen), ptr(cnt), ptr(fl)))
