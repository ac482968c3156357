"""ctypes wrapper over oracle/build/liboracle.so — TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this
module, and only as the checker (or as the timed CPU baseline).  The product
(libdmf.so + dmf_amd) never imports it.

PARITY UNPINNED: the reference ships no golden vectors and cannot be built here
(see oracle.cpp header and DESIGN.md §2).  Each method names the reference
function it restates (file:line under the reference tree).
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "build", "liboracle.so")
_lib = None

_f32p = np.ctypeslib.ndpointer(np.float32, flags="C_CONTIGUOUS")
_u16p = np.ctypeslib.ndpointer(np.uint16, flags="C_CONTIGUOUS")
_i32p = np.ctypeslib.ndpointer(np.int32, flags="C_CONTIGUOUS")
_i16p = np.ctypeslib.ndpointer(np.int16, flags="C_CONTIGUOUS")
_u64p = np.ctypeslib.ndpointer(np.uint64, flags="C_CONTIGUOUS")
_i64p = np.ctypeslib.ndpointer(np.int64, flags="C_CONTIGUOUS")
_u8p = np.ctypeslib.ndpointer(np.uint8, flags="C_CONTIGUOUS")
_f64p = np.ctypeslib.ndpointer(np.float64, flags="C_CONTIGUOUS")
_vp = C.c_void_p


def build():
    """Compile liboracle.so with the committed Makefile (g++ only)."""
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def lib():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(_LIB_PATH):
        build()
    L = C.CDLL(_LIB_PATH)
    sig = {
        "orc_volume_new": (_vp, []),
        "orc_volume_free": (None, [_vp]),
        "orc_set_dimensions": (None, [_vp] + [C.c_double] * 6),
        "orc_set_resolution": (None, [_vp] + [C.c_double] * 3),
        "orc_set_volume_size": (None, [_vp] + [C.c_int] * 3),
        "orc_construct": (C.c_int, [_vp]),
        "orc_get_info": (None, [_vp, _f64p, _i32p, _u64p]),
        "orc_hazards": (C.c_int64, [_vp]),
        "orc_integrate": (C.c_int64, [_vp, _f32p, _vp, C.c_int64]),
        "orc_num_occupied": (C.c_int64, [_vp]),
        "orc_occupied": (C.c_int64, [_vp, _u64p, C.c_int64]),
        "orc_voxel_table": (None, [_vp, _i32p, _u8p, _i64p, _i64p]),
        "orc_voxel_points": (C.c_int64, [_vp, C.c_int, C.c_int, C.c_int, _f32p, _f32p, C.c_int64]),
        "orc_reset_flags": (None, [_vp]),
        "orc_occupancy_dense": (None, [_vp, _u8p]),
        "orc_project_point": (None, [_f32p, C.c_int, C.c_int, C.c_int, _f32p]),
        "orc_deproject_point": (None, [_f32p, C.c_double, C.c_double, C.c_double, _i32p]),
        "orc_transform_point": (None, [_f32p, C.c_double, C.c_double, C.c_double, _f32p]),
        "orc_inverse_pose": (None, [_f32p, _f32p]),
        "orc_degree": (C.c_int, [C.c_double]),
        "orc_angle_ok": (C.c_int, [_f32p, _f32p]),
        "orc_backproject": (None, [_f32p, C.c_int, C.c_int, _u16p, _f32p, _f32p]),
        "orc_reverse_ray_trace_fast": (C.c_int64, [_vp, _f32p, C.c_int, C.c_int, _f32p, C.c_int, C.c_int,
                                                   C.POINTER(C.c_int), _u64p, C.c_int64]),
        "orc_reverse_ray_trace": (C.c_int64, [_vp, _f32p, C.c_int, C.c_int, _f32p, C.c_int,
                                              C.POINTER(C.c_int), _u64p, C.c_int64]),
        "orc_float_axis": (C.c_int64, [C.c_double, C.c_double, C.c_double, _f32p, C.c_int64]),
        "orc_ray_trace": (None, [_vp, _f32p, C.c_int, C.c_int, _f32p, C.c_int, C.c_int]),
        "orc_ray_trace_and_classify": (None, [_vp, _f32p, C.c_int, C.c_int, _f32p, C.c_int, C.c_int, C.c_int]),
        "orc_ray_trace_and_get_good_points": (C.c_int64, [_vp, _f32p, C.c_int, C.c_int, _f32p, C.c_int, C.c_int,
                                                          C.POINTER(C.c_int), _u64p, C.c_int64]),
        "orc_ray_trace_and_get_points": (C.c_int64, [_vp, _f32p, C.c_int, C.c_int, _f32p, C.c_int, C.c_int,
                                                     C.POINTER(C.c_int), _u64p, C.c_int64]),
        "orc_ray_trace_and_get_minimum": (C.c_int, [_vp, _f32p, C.c_int, C.c_int, _f32p, C.c_int, C.c_int]),
        "orc_forward_first_hits": (None, [_vp, _f32p, C.c_int, C.c_int, _f32p, C.c_int, C.c_int, C.c_int,
                                          C.c_int, _i32p, _u64p]),
        "orc_ray_trace_volume": (None, [_vp, _f32p, C.c_int, C.c_int, _f32p, _i32p]),
        "orc_will_collide": (C.c_int, [_vp, _f32p, _f32p]),
        "orc_collision_cost_map": (None, [_vp, _f32p, C.c_int, _i32p]),
        "orc_fuse_depth": (None, [_vp, _f32p, C.c_int, C.c_int, _u16p, _f32p, C.c_int, C.c_int, C.c_int,
                                  _i32p, _i32p, _i64p]),
        "orc_fuse_finalize": (None, [C.c_int64, _i32p, _i32p, C.c_int, C.c_int, C.c_int, C.c_int, _i16p]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args
    _lib = L
    return L


def _f32(a, n=None):
    a = np.ascontiguousarray(a, dtype=np.float32)
    if n is not None:
        assert a.size == n, (a.shape, n)
    return a


# --------------------------------------------------------------------------- camera
def project_point(K, r, c, d):
    """Camera.hpp:24-31 projectPoint."""
    out = np.zeros(3, np.float32)
    lib().orc_project_point(_f32(K, 9), r, c, d, out)
    return out


def deproject_point(K, x, y, z):
    """Camera.hpp:32-38 deProjectPoint -> (r, c)."""
    rc = np.zeros(2, np.int32)
    lib().orc_deproject_point(_f32(K, 9), float(x), float(y), float(z), rc)
    return int(rc[0]), int(rc[1])


def transform_point(T, x, y, z):
    """Camera.hpp:39-45 transformPoints."""
    out = np.zeros(3, np.float32)
    lib().orc_transform_point(_f32(T, 12), float(x), float(y), float(z), out)
    return out


def inverse_pose(T):
    """Eigen Affine3f::inverse() as used at RayTracingEngine.hpp:140."""
    out = np.zeros(12, np.float32)
    lib().orc_inverse_pose(_f32(T, 12), out)
    return out


def degree(rad):
    """CommonUtilities.hpp:17."""
    return lib().orc_degree(float(rad))


def angle_ok(n, v):
    return bool(lib().orc_angle_ok(_f32(n, 3), _f32(v, 3)))


def backproject(K, depth, T):
    """Camera.hpp:24-45 per pixel: projectPoint then transformPoints -> (H, W, 3) float32."""
    depth = np.ascontiguousarray(depth, np.uint16)
    H, W = depth.shape
    out = np.zeros((H, W, 3), np.float32)
    lib().orc_backproject(_f32(K, 9), H, W, depth, _f32(T, 12), out)
    return out


def float_axis(lo, hi, delta):
    """`for(float x=lo; x<hi; x+=delta)` sequence (RayTracingEngine.hpp:54)."""
    n = lib().orc_float_axis(lo, hi, delta, np.zeros(1, np.float32), 0)
    out = np.zeros(max(n, 1), np.float32)
    lib().orc_float_axis(lo, hi, delta, out, n)
    return out[:n]


# --------------------------------------------------------------------------- volume
class Volume:
    """Volume.hpp:50-255 VoxelVolume, reference layout (pointer grid)."""

    def __init__(self):
        self._h = lib().orc_volume_new()

    def __del__(self):
        if getattr(self, "_h", None):
            lib().orc_volume_free(self._h)
            self._h = None

    def setDimensions(self, xmin, xmax, ymin, ymax, zmin, zmax):
        lib().orc_set_dimensions(self._h, xmin, xmax, ymin, ymax, zmin, zmax)

    def setResolution(self, dx, dy, dz):
        lib().orc_set_resolution(self._h, dx, dy, dz)

    def setVolumeSize(self, nx, ny, nz):
        lib().orc_set_volume_size(self._h, nx, ny, nz)

    def constructVolume(self):
        return bool(lib().orc_construct(self._h))

    def info(self):
        d = np.zeros(13, np.float64)
        dims = np.zeros(3, np.int32)
        hs = np.zeros(1, np.uint64)
        lib().orc_get_info(self._h, d, dims, hs)
        keys = ["xmin_", "xmax_", "ymin_", "ymax_", "zmin_", "zmax_", "xcenter_", "ycenter_", "zcenter_",
                "xdelta_", "ydelta_", "zdelta_", "voxel_size_"]
        out = dict(zip(keys, d.tolist()))
        out.update(xdim_=int(dims[0]), ydim_=int(dims[1]), zdim_=int(dims[2]), hsize_=int(hs[0]))
        return out

    @property
    def dims(self):
        i = self.info()
        return i["xdim_"], i["ydim_"], i["zdim_"]

    def hazards(self):
        return lib().orc_hazards(self._h)

    def integratePointCloud(self, xyz, normals=None):
        """Volume.hpp:172-228. Returns number of points binned."""
        xyz = _f32(xyz).reshape(-1, 3)
        nrm = None
        if normals is not None:
            nrm = _f32(normals).reshape(-1, 3)
            assert nrm.shape == xyz.shape
        return lib().orc_integrate(self._h, xyz, None if nrm is None else nrm.ctypes.data, xyz.shape[0])

    @property
    def occupied_cells_(self):
        n = lib().orc_num_occupied(self._h)
        out = np.zeros(max(n, 1), np.uint64)
        lib().orc_occupied(self._h, out, n)
        return out[:n]

    def voxel_table(self):
        """(view int32, good uint8, npts int64, nnormals int64) in occupied_cells_ order."""
        n = lib().orc_num_occupied(self._h)
        view = np.zeros(max(n, 1), np.int32)
        good = np.zeros(max(n, 1), np.uint8)
        npts = np.zeros(max(n, 1), np.int64)
        nn = np.zeros(max(n, 1), np.int64)
        lib().orc_voxel_table(self._h, view, good, npts, nn)
        return view[:n], good[:n], npts[:n], nn[:n]

    def voxel_points(self, x, y, z):
        n = lib().orc_voxel_points(self._h, x, y, z, np.zeros(3, np.float32), np.zeros(3, np.float32), 0)
        if n < 0:
            return None, None
        p = np.zeros((max(n, 1), 3), np.float32)
        q = np.zeros((max(n, 1), 3), np.float32)
        lib().orc_voxel_points(self._h, x, y, z, p, q, n)
        return p[:n], q[:n]

    def reset_flags(self):
        lib().orc_reset_flags(self._h)

    def occupancy_dense(self):
        nx, ny, nz = self.dims
        out = np.zeros(nx * ny * nz, np.uint8)
        lib().orc_occupancy_dense(self._h, out)
        return out.reshape(nx, ny, nz)


# --------------------------------------------------------------------------- engine
def _list_call(fn, *args):
    found = C.c_int(0)
    n = fn(*args, C.byref(found), np.zeros(1, np.uint64), 0)
    out = np.zeros(max(n, 1), np.uint64)
    fn(*args, C.byref(found), out, n)
    return bool(found.value), out[:n]


def _list_call_mut(vol, fn, *args):
    # list-returning calls that also mutate flags: run once into a big-enough buffer
    found = C.c_int(0)
    cap = max(int(lib().orc_num_occupied(vol._h)) * 2 + 16, 1 << 16)
    while True:
        out = np.zeros(cap, np.uint64)
        n = fn(vol._h, *args, C.byref(found), out, cap)
        if n <= cap:
            return bool(found.value), out[:n]
        cap = n  # flags are idempotent, a re-run gives the same result


class Engine:
    """RayTracingEngine.hpp:27-40 over a Camera(K, height, width)."""

    def __init__(self, K, height=480, width=640):
        self.K = _f32(K, 9)
        self.H = height
        self.W = width

    def reverseRayTraceFast(self, vol, T, viz, zdelta=1, dead_work=False):
        """RayTracingEngine.hpp:136-226."""
        return _list_call_mut(vol, lib().orc_reverse_ray_trace_fast, self.K, self.H, self.W, _f32(T, 12),
                              int(bool(viz)), int(bool(dead_work)))

    def reverseRayTrace(self, vol, T, viz, zdelta=1):
        """RayTracingEngine.hpp:45-134."""
        return _list_call_mut(vol, lib().orc_reverse_ray_trace, self.K, self.H, self.W, _f32(T, 12),
                              int(bool(viz)))

    def rayTrace(self, vol, T, zdelta=10, sparse=True):
        lib().orc_ray_trace(vol._h, self.K, self.H, self.W, _f32(T, 12), zdelta, int(bool(sparse)))

    def rayTraceAndClassify(self, vol, T, zdelta=10, view=1, sparse=True):
        lib().orc_ray_trace_and_classify(vol._h, self.K, self.H, self.W, _f32(T, 12), zdelta, view,
                                         int(bool(sparse)))

    def rayTraceAndGetGoodPoints(self, vol, T, zdelta=10, sparse=True):
        return _list_call_mut(vol, lib().orc_ray_trace_and_get_good_points, self.K, self.H, self.W,
                              _f32(T, 12), zdelta, int(bool(sparse)))

    def rayTraceAndGetPoints(self, vol, T, zdelta=10, sparse=True):
        return _list_call_mut(vol, lib().orc_ray_trace_and_get_points, self.K, self.H, self.W,
                              _f32(T, 12), zdelta, int(bool(sparse)))

    def rayTraceAndGetMinimum(self, vol, T, zdelta=1, sparse=True):
        return lib().orc_ray_trace_and_get_minimum(vol._h, self.K, self.H, self.W, _f32(T, 12), zdelta,
                                                   int(bool(sparse)))

    def rayTraceVolume(self, vol, T):
        depth = np.zeros(self.H * self.W, np.int32)
        lib().orc_ray_trace_volume(vol._h, self.K, self.H, self.W, _f32(T, 12), depth)
        return depth.reshape(self.H, self.W)

    def forward_first_hits(self, vol, T, zstart, zdelta, rdelta, cdelta):
        R = (self.H + rdelta - 1) // rdelta
        Cc = (self.W + cdelta - 1) // cdelta
        k = np.zeros(R * Cc, np.int32)
        h = np.zeros(R * Cc, np.uint64)
        lib().orc_forward_first_hits(vol._h, self.K, self.H, self.W, _f32(T, 12), zstart, zdelta, rdelta,
                                     cdelta, k, h)
        return k.reshape(R, Cc), h.reshape(R, Cc)


def will_collide(vol, a, b):
    """tests/CameraPathGen.cpp:128-156."""
    return bool(lib().orc_will_collide(vol._h, _f32(a, 3), _f32(b, 3)))


def collision_cost_map(vol, poses):
    """tests/CameraPathGen.cpp:310-331 run_tsp cost map: (V, V) int32, INT_MAX = collided."""
    poses = np.ascontiguousarray(poses, np.float32).reshape(-1, 12)
    V = poses.shape[0]
    out = np.zeros((V, V), np.int32)
    lib().orc_collision_cost_map(vol._h, _f32(poses, 12 * V), V, out)
    return out


# --------------------------------------------------------------------------- fusion (own spec)
LOGODDS_DEFAULT = dict(l_hit=847, l_miss=-405, l_min=-2000, l_max=3511)


def fuse_depth(vol, K, depth, poses, dmin=1, dmax=65535, hits=None, misses=None, threads=1):
    """DESIGN.md §4 3D-DDA fusion of P depth frames.  depth (P,H,W) uint16, poses (P,12).
    threads > 1: the OpenMP row-parallel variant (same counts)."""
    depth = np.ascontiguousarray(depth, np.uint16)
    if depth.ndim == 2:
        depth = depth[None]
    P, H, W = depth.shape
    poses = _f32(poses).reshape(P, 12)
    n = int(np.prod(vol.dims))
    if hits is None:
        hits = np.zeros(n, np.int32)
    if misses is None:
        misses = np.zeros(n, np.int32)
    stats = np.zeros(3, np.int64)
    if threads > 1:
        L = lib()
        L.orc_fuse_depth_mt.restype = None
        L.orc_fuse_depth_mt.argtypes = list(L.orc_fuse_depth.argtypes) + [C.c_int]
        L.orc_fuse_depth_mt(vol._h, _f32(K, 9), H, W, depth, poses, P, dmin, dmax, hits, misses, stats, int(threads))
    else:
        lib().orc_fuse_depth(vol._h, _f32(K, 9), H, W, depth, poses, P, dmin, dmax, hits, misses, stats)
    return hits, misses, stats


def greedy_set_cover(sets, min_gain=5):
    """Algorithms.hpp:38-86 greedySetCover over sorted hash lists -> selected ids."""
    sets = [np.sort(np.asarray(x, np.uint64)) for x in sets]
    counts = np.array([len(x) for x in sets], np.int64)
    flat = np.concatenate(sets) if len(sets) and counts.sum() else np.zeros(1, np.uint64)
    out = np.zeros(max(len(sets), 1), np.int32)
    L = lib()
    L.orc_greedy_set_cover.restype = C.c_int32
    L.orc_greedy_set_cover.argtypes = [_u64p, _i64p, C.c_int32, C.c_int32, _i32p]
    n = L.orc_greedy_set_cover(flat, counts, len(sets), int(min_gain), out)
    return out[:n]


def fuse_finalize(hits, misses, l_hit=847, l_miss=-405, l_min=-2000, l_max=3511):
    out = np.zeros(hits.size, np.int16)
    lib().orc_fuse_finalize(hits.size, np.ascontiguousarray(hits, np.int32),
                            np.ascontiguousarray(misses, np.int32), l_hit, l_miss, l_min, l_max, out)
    return out


class OccupancyGrid:
    """OccupancyGrid.hpp:50-318 restated (sequential order), dense state."""

    def __init__(self):
        L = lib()
        for name, res, args in (("orc_ogrid_new", _vp, []), ("orc_ogrid_free", None, [_vp]),
                                ("orc_ogrid_setup", None, [_vp, _f64p, C.c_float, C.c_float, C.c_float, C.c_int]),
                                ("orc_ogrid_dims", None, [_vp, _i32p]),
                                ("orc_ogrid_update", None, [_vp, _f32p, C.c_int64, _f32p, C.c_int64]),
                                ("orc_ogrid_state", None, [_vp, _f32p, _f32p, _i32p, _u8p]),
                                ("orc_ogrid_download", C.c_int64, [_vp, C.c_int, _f32p, C.c_int64]),
                                ("orc_ogrid_set_state", None, [_vp, _f32p, _f32p, _i32p, _u8p]),
                                ("orc_ogrid_download_reorganized", C.c_int64, [_vp, C.c_int, _f32p, C.c_int64])):
            fn = getattr(L, name)
            fn.restype, fn.argtypes = res, args
        self._L = L
        self._h = L.orc_ogrid_new()
        self._b = None
        self._r = None
        self._k = 0

    def __del__(self):
        if getattr(self, "_h", None):
            self._L.orc_ogrid_free(self._h)
            self._h = None

    def setDimensions(self, xmin, xmax, ymin, ymax, zmin, zmax):
        self._b = np.array([xmin, xmax, ymin, ymax, zmin, zmax], np.float64)

    def setResolution(self, x, y, z):
        self._r = (np.float32(x), np.float32(y), np.float32(z))

    def setK(self, k):
        self._k = int(k)

    def construct(self):
        self._L.orc_ogrid_setup(self._h, self._b, *self._r, self._k)
        return True

    @property
    def dims(self):
        d = np.zeros(3, np.int32)
        self._L.orc_ogrid_dims(self._h, d)
        return tuple(int(x) for x in d)

    def updateStates(self, cloud, normals):
        cloud = np.ascontiguousarray(cloud, np.float32).reshape(-1, 3)
        normals = np.ascontiguousarray(normals, np.float32).reshape(-1, 6)
        self._L.orc_ogrid_update(self._h, cloud, cloud.shape[0], normals, normals.shape[0])
        return True

    def state(self):
        n = int(np.prod(self.dims))
        nrm, cen = np.zeros(3 * n, np.float32), np.zeros(3 * n, np.float32)
        cnt, fl = np.zeros(n, np.int32), np.zeros(n, np.uint8)
        self._L.orc_ogrid_state(self._h, nrm, cen, cnt, fl)
        return nrm.reshape(-1, 3), cen.reshape(-1, 3), cnt, fl

    def download(self, mode=0):
        n = self._L.orc_ogrid_download(self._h, mode, np.zeros(6, np.float32), 0)
        out = np.zeros(6 * max(n, 1), np.float32)
        self._L.orc_ogrid_download(self._h, mode, out, n)
        return out[:6 * n].reshape(-1, 6)

    def set_state(self, normal, centroid, count, flags):
        """Write the dense voxels_ fields (normal, centroid: (n, 3) float; count int32;
        flags: occupied | normal_found << 1)."""
        n = int(np.prod(self.dims))
        self._L.orc_ogrid_set_state(self._h, np.ascontiguousarray(normal, np.float32).reshape(3 * n),
                                    np.ascontiguousarray(centroid, np.float32).reshape(3 * n),
                                    np.ascontiguousarray(count, np.int32).reshape(n),
                                    np.ascontiguousarray(flags, np.uint8).reshape(n))

    def downloadReorganizedCloud(self, clean=False):
        """OccupancyGrid.hpp:200-286, single-threaded order."""
        n = self._L.orc_ogrid_download_reorganized(self._h, int(bool(clean)), np.zeros(6, np.float32), 0)
        out = np.zeros(6 * max(n, 1), np.float32)
        self._L.orc_ogrid_download_reorganized(self._h, int(bool(clean)), out, n)
        return out[:6 * n].reshape(-1, 6)
