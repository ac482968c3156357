"""ctypes binding of libdmf.so (include/dmf.h).

The shared library is the product: there is no Python or CPU fallback.  If the
library is missing or no gfx950 GPU is visible, every compute call raises.

Import order: when PyTorch is used in the same process, import torch BEFORE
loading this library so both share torch's HIP runtime (same soname
libamdhip64.so.7); see INTEGRATION.md.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

PKG_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.environ.get("DMF_LIB", os.path.join(PKG_ROOT, "build", "libdmf.so"))
REPO_ROOT = os.path.dirname(PKG_ROOT)
HEADER_PATH = os.path.join(REPO_ROOT, "include", "dmf.h")
DIAG_HEADER_PATH = os.path.join(REPO_ROOT, "include", "dmf_diag.h")

DMF_OK = 0
DMF_ERR_INVALID = 1
DMF_ERR_STATE = 2
DMF_ERR_HIP = 3
DMF_ERR_NOMEM = 4
DMF_ERR_CAPACITY = 5
DMF_ERR_RANGE = 6
DMF_ERR_NO_DEVICE = 7
DMF_ERR_DEVICE_CHECK = 8


class DmfError(RuntimeError):
    def __init__(self, status, msg):
        super().__init__(f"dmf status {status}: {msg}")
        self.status = status


class dmf_camera(C.Structure):
    _fields_ = [("K", C.c_float * 9), ("height", C.c_int32), ("width", C.c_int32)]


class dmf_volume_info(C.Structure):
    _fields_ = [(n, C.c_double) for n in ("xmin", "xmax", "ymin", "ymax", "zmin", "zmax", "xcenter", "ycenter",
                                          "zcenter", "xdelta", "ydelta", "zdelta", "voxel_size")] + [
        ("xdim", C.c_int32), ("ydim", C.c_int32), ("zdim", C.c_int32), ("constructed", C.c_int32),
        ("hsize", C.c_uint64), ("num_occupied", C.c_int64), ("num_points", C.c_int64), ("hazards", C.c_int64)]


class dmf_fuse_plan_info(C.Structure):
    _fields_ = [("brick", C.c_int32), ("max_batches", C.c_int32), ("poses_per_batch", C.c_int32),
                ("record_bytes", C.c_int32), ("pair_capacity", C.c_uint64), ("scratch_bytes", C.c_uint64),
                ("super_batch_poses", C.c_int32), ("slots", C.c_int32)]


class dmf_merge_plan(C.Structure):
    _fields_ = [(n, C.c_int64) for n in ("n_padded", "chunk", "chunk_offset", "tile_begin", "tile_end",
                                         "logodds_padded", "slab_bytes", "slab_offset")]


class dmf_fuse_params(C.Structure):
    _fields_ = [("dmin_mm", C.c_int32), ("dmax_mm", C.c_int32), ("l_hit", C.c_int32), ("l_miss", C.c_int32),
                ("l_min", C.c_int32), ("l_max", C.c_int32)]


class dmf_grid_header(C.Structure):
    _fields_ = [("dims", C.c_int32 * 3), ("reserved", C.c_int32), ("bounds", C.c_double * 6),
                ("params", dmf_fuse_params)]


_vp = C.c_void_p
_p = C.c_void_p  # raw pointers are passed as integers (numpy .ctypes.data or device addresses)
_i32 = C.c_int32
_i64 = C.c_int64

SIGNATURES = {
    "dmf_abi_version": (C.c_int, []),
    "dmf_status_string": (C.c_char_p, [C.c_int]),
    "dmf_last_error": (C.c_char_p, []),
    "dmf_device_count": (C.c_int, [_p]),
    "dmf_fuse_params_default": (None, [_p]),
    "dmf_angle_threshold": (C.c_int, [_p]),
    "dmf_fuse_kernel_name": (C.c_char_p, [_vp]),
    "dmf_fuse_set_variant": (C.c_int, [_vp, _i32]),
    "dmf_fuse_get_variant": (C.c_int, [_vp, _p]),
    "dmf_volume_set_knob": (C.c_int, [_vp, _i32, _i64]),
    "dmf_volume_get_knob": (C.c_int, [_vp, _i32, _p]),
    "dmf_volume_create": (C.c_int, [_p, _i32]),
    "dmf_volume_destroy": (C.c_int, [_vp]),
    "dmf_volume_set_stream": (C.c_int, [_vp, _vp]),
    "dmf_volume_synchronize": (C.c_int, [_vp]),
    "dmf_volume_set_dimensions": (C.c_int, [_vp] + [C.c_double] * 6),
    "dmf_volume_set_resolution": (C.c_int, [_vp] + [C.c_double] * 3),
    "dmf_volume_set_volume_size": (C.c_int, [_vp, _i32, _i32, _i32]),
    "dmf_volume_construct": (C.c_int, [_vp]),
    "dmf_volume_get_info": (C.c_int, [_vp, _p]),
    "dmf_volume_integrate": (C.c_int, [_vp, _p, _p, _i64, _p, _p]),
    "dmf_volume_integrate_device": (C.c_int, [_vp, _p, _p, _i64]),
    "dmf_volume_occupied": (C.c_int, [_vp, _p, _i64, _p]),
    "dmf_volume_voxel_flags": (C.c_int, [_vp, _p, _p, _i64]),
    "dmf_volume_reset_flags": (C.c_int, [_vp]),
    "dmf_volume_voxel_counts": (C.c_int, [_vp, _p, _p, _i64]),
    "dmf_volume_voxel_points": (C.c_int, [_vp, C.c_uint64, _p, _p, _i64, _p]),
    "dmf_volume_occupancy": (C.c_int, [_vp, _p]),
    "dmf_volume_export": (C.c_int, [_vp, _p, _p, _p, _i64]),
    "dmf_backproject": (C.c_int, [_vp, _p, _p, _p, _p]),
    "dmf_backproject_device": (C.c_int, [_vp, _p, _p, _p, _i32, _p]),
    "dmf_reverse_ray_trace_fast": (C.c_int, [_vp, _p, _p, _i32, _i32, _p, _p, _p, _i64]),
    "dmf_reverse_visibility_device": (C.c_int, [_vp, _p, _p, _i32, _i32, _p, _p, _p]),
    "dmf_reverse_ray_trace": (C.c_int, [_vp, _p, _p, _i32, _i32, _p, _p, _p, _i64]),
    "dmf_ray_trace": (C.c_int, [_vp, _p, _p, _i32, _i32]),
    "dmf_ray_trace_and_classify": (C.c_int, [_vp, _p, _p, _i32, _i32, _i32]),
    "dmf_ray_trace_and_get_minimum": (C.c_int, [_vp, _p, _p, _i32, _i32, _p]),
    "dmf_ray_trace_and_get_points": (C.c_int, [_vp, _p, _p, _i32, _i32, _p, _p, _i64, _p]),
    "dmf_ray_trace_and_get_good_points": (C.c_int, [_vp, _p, _p, _i32, _i32, _p, _p, _i64, _p]),
    "dmf_forward_first_hits": (C.c_int, [_vp, _p, _p, _i32, _i32, _i32, _i32, _p, _p]),
    "dmf_ray_trace_volume": (C.c_int, [_vp, _p, _p, _p]),
    "dmf_will_collide": (C.c_int, [_vp, _p, _p, _i64, _p]),
    "dmf_collision_cost_map": (C.c_int, [_vp, _p, _i32, _p]),
    "dmf_collision_cost_map_device": (C.c_int, [_vp, _p, _i32, _p]),
    "dmf_forward_first_hits_device": (C.c_int, [_vp, _p, _p, _i32, _i32, _i32, _i32, _i32, _p, _p, _p]),
    "dmf_greedy_set_cover": (C.c_int, [_vp, _p, _p, _i32, _i32, _p, _p]),
    "dmf_greedy_set_cover_masks_device": (C.c_int, [_vp, _p, _i32, _i64, _i32, _p, _p]),
    "dmf_fuse_depth": (C.c_int, [_vp, _p, _p, _p, _i32, _p, _p, _p, _p]),
    "dmf_fuse_depth_device": (C.c_int, [_vp, _p, _p, _p, _i32, _p, _p, _p, _p]),
    "dmf_fuse_finalize": (C.c_int, [_vp, _p, _p, _p, _p]),
    "dmf_fuse_finalize_device": (C.c_int, [_vp, _p, _p, _p, _p]),
    "dmf_fuse_counter_cells": (C.c_int, [_vp, _p]),
    "dmf_fuse_counters_to_linear_device": (C.c_int, [_vp, _p, _p]),
    "dmf_fuse_reserve": (C.c_int, [_vp, _p, _i32, C.c_uint64]),
    "dmf_fuse_set_input_stream": (C.c_int, [_vp, _vp]),
    "dmf_fuse_set_phase_event": (C.c_int, [_vp, _vp]),
    "dmf_fuse_plan": (C.c_int, [_vp, _p, _i32, _p]),
    "dmf_grid_save": (C.c_int, [C.c_char_p, _p, _p]),
    "dmf_grid_load": (C.c_int, [C.c_char_p, _p, _p, _i64]),
    "dmf_fuse_batches_used": (C.c_int, [_vp, _p]),
    "dmf_fuse_status": (C.c_int, [_vp, _p]),
    "dmf_rccl_version": (C.c_int, [_p]),
    "dmf_comm_unique_id": (C.c_int, [_p]),
    "dmf_comm_init_rank": (C.c_int, [_p, _i32, _p, _i32, _i32]),
    "dmf_comm_destroy": (C.c_int, [_vp]),
    "dmf_comm_shape": (C.c_int, [_vp, _p, _p]),
    "dmf_fuse_counter_cells_padded": (C.c_int, [_vp, _i32, _p]),
    "dmf_fuse_logodds_cells_padded": (C.c_int, [_vp, _i32, _p]),
    "dmf_fuse_allreduce_device": (C.c_int, [_vp, _p, _i64, _vp, _vp]),
    "dmf_fuse_merge_plan": (C.c_int, [_vp, _i32, _i32, _p]),
    "dmf_fuse_merge_plan_dims": (C.c_int, [_i32, _i32, _i32, _i32, _i32, _p]),
    "dmf_fuse_finalize_slab_device": (C.c_int, [_vp, _p, _p, _p, _i32, _i32, _vp]),
    "dmf_fuse_merge_finalize_device": (C.c_int, [_vp, _p, _p, _p, _vp, _vp]),
    "dmf_flags_allreduce": (C.c_int, [_vp, _vp, _vp]),
    "dmf_ogrid_create": (C.c_int, [_p, _i32]),
    "dmf_ogrid_destroy": (C.c_int, [_vp]),
    "dmf_ogrid_set_stream": (C.c_int, [_vp, _vp]),
    "dmf_ogrid_setup": (C.c_int, [_vp, _p, C.c_float, C.c_float, C.c_float, _i32]),
    "dmf_ogrid_get_dims": (C.c_int, [_vp, _p]),
    "dmf_ogrid_update_states": (C.c_int, [_vp, _p, _i64, _p, _i64]),
    "dmf_ogrid_update_states_device": (C.c_int, [_vp, _p, _i64, _p, _i64]),
    "dmf_ogrid_state": (C.c_int, [_vp, _p, _p, _p, _p]),
    "dmf_ogrid_download": (C.c_int, [_vp, _i32, _p, _i64, _p]),
    "dmf_ogrid_set_state": (C.c_int, [_vp, _p, _p, _p, _p]),
    "dmf_device_malloc": (C.c_int, [_vp, _p, C.c_size_t]),
    "dmf_device_free": (C.c_int, [_vp, _vp]),
    "dmf_memcpy_h2d": (C.c_int, [_vp, _vp, _p, C.c_size_t]),
    "dmf_memcpy_d2h": (C.c_int, [_vp, _p, _vp, C.c_size_t]),
    "dmf_memset_device": (C.c_int, [_vp, _vp, C.c_int, C.c_size_t]),
}

_lib = None


def load(path=None):
    """Load libdmf.so (raises if it has not been built: no fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    path = path or LIB_PATH
    if not os.path.exists(path):
        raise ImportError(f"libdmf.so not found at {path}; run `make -C depth-map-fusion-utils_amd` "
                          "(or __graft_entry__.build()).  There is no CPU fallback.")
    L = C.CDLL(path)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args
    _lib = L
    return L


def check(status):
    if status != DMF_OK:
        L = load()
        raise DmfError(status, f"{L.dmf_status_string(status).decode()}: {L.dmf_last_error().decode()}")
    return status


def ptr(a):
    """Raw address of a numpy array (or None)."""
    if a is None:
        return None
    return a.ctypes.data


def device_count():
    n = C.c_int32(0)
    check(load().dmf_device_count(C.addressof(n)))
    return n.value


def declared_symbols():
    """Function names declared in include/dmf.h and include/dmf_diag.h (parsed from the
    header text)."""
    import re
    txt = open(HEADER_PATH).read() + open(DIAG_HEADER_PATH).read()
    return sorted(set(re.findall(r"\b(dmf_[a-z0-9_]+)\s*\(", txt)))


# include/dmf_diag.h: fusion implementations and per-volume knobs (diagnostics, A/B, tests)
FUSE_DEFAULT, FUSE_LDS_BOX, FUSE_CELL_WALK, FUSE_SLAB = 0, 31, 40, 57
KNOBS = {"super_poses": 1, "pair_cap": 2, "batch_poses": 3, "part_max": 4, "span": 5, "tail_split": 6,
         "reverse_kernel": 7, "fwd_skip": 8, "a_hash": 9, "fault_inject": 10, "fwd_kernel": 11,
         "bdist_cap": 12}


def fuse_status(vol):
    """dmf_fuse_status: raises DmfError (DMF_ERR_DEVICE_CHECK) when a fusion call of this volume
    since the last check failed the device-side pair-layout check; returns the fault count (0)."""
    f = C.c_uint64(0)
    check(load().dmf_fuse_status(getattr(vol, "_h", vol), C.addressof(f)))
    return f.value


def set_variant(vol, variant):
    """dmf_fuse_set_variant on a dmf_amd.VoxelVolume (or a raw handle)."""
    check(load().dmf_fuse_set_variant(getattr(vol, "_h", vol), int(variant)))


def kernel_name(vol):
    """dmf_fuse_kernel_name: the fusion kernel of the volume's latest call."""
    return load().dmf_fuse_kernel_name(getattr(vol, "_h", vol)).decode()


def set_knob(vol, name, value):
    """dmf_volume_set_knob by name (KNOBS); 0 = the default."""
    check(load().dmf_volume_set_knob(getattr(vol, "_h", vol), KNOBS[name], int(value)))


def make_camera(K, height=480, width=640):
    cam = dmf_camera()
    Kf = np.asarray(K, np.float32).reshape(9)
    for i in range(9):
        cam.K[i] = float(Kf[i])
    cam.height = int(height)
    cam.width = int(width)
    return cam


def default_fuse_params(**kw):
    p = dmf_fuse_params()
    load().dmf_fuse_params_default(C.addressof(p))
    for k, v in kw.items():
        setattr(p, k, int(v))
    return p


def fuse_plan(vol, cam, P):
    """dmf_fuse_plan of a fusion call of P frames of `cam` (a dmf_camera) on `vol` (a
    dmf_amd.VoxelVolume) as a dict."""
    info = dmf_fuse_plan_info()
    check(load().dmf_fuse_plan(vol._h, C.addressof(cam), int(P), C.addressof(info)))
    return {k: getattr(info, k) for k, _ in dmf_fuse_plan_info._fields_}


def merge_plan(vol, nranks, rank):
    """dmf_fuse_merge_plan as a dict (rank = -1: the whole grid)."""
    out = dmf_merge_plan()
    check(load().dmf_fuse_merge_plan(vol._h, int(nranks), int(rank), C.addressof(out)))
    return {k: getattr(out, k) for k, _ in dmf_merge_plan._fields_}


def merge_plan_dims(dims, nranks, rank):
    """dmf_fuse_merge_plan_dims (host only) as a dict."""
    out = dmf_merge_plan()
    check(load().dmf_fuse_merge_plan_dims(int(dims[0]), int(dims[1]), int(dims[2]), int(nranks), int(rank),
                                          C.addressof(out)))
    return {k: getattr(out, k) for k, _ in dmf_merge_plan._fields_}


def fuse_batches_used(vol):
    """dmf_fuse_batches_used: pose batches of the latest brick-pipeline super-batch."""
    n = C.c_int32()
    check(load().dmf_fuse_batches_used(vol._h, C.addressof(n)))
    return n.value


def grid_save(path, logodds, dims, bounds, params=None):
    """dmf_grid_save: the int16 log-odds grid (x-major, dims cells) with its geometry and
    fusion parameters (dmf_fuse_params; None = the defaults) to `path`."""
    lo = np.ascontiguousarray(logodds, np.int16).reshape(-1)
    if lo.size != int(np.prod(dims)):
        raise ValueError(f"logodds has {lo.size} cells, dims {tuple(dims)} need {int(np.prod(dims))}")
    h = dmf_grid_header()
    for a in range(3):
        h.dims[a] = int(dims[a])
    for i in range(6):
        h.bounds[i] = float(bounds[i])
    h.params = params if params is not None else default_fuse_params()
    check(load().dmf_grid_save(os.fsencode(str(path)), C.addressof(h), lo.ctypes.data))


def grid_load(path):
    """dmf_grid_load -> (logodds int16 (x, y, z), bounds tuple, dmf_fuse_params)."""
    h = dmf_grid_header()
    L = load()
    check(L.dmf_grid_load(os.fsencode(str(path)), C.addressof(h), None, 0))
    dims = tuple(int(h.dims[a]) for a in range(3))
    out = np.empty(int(np.prod(dims)), np.int16)
    check(L.dmf_grid_load(os.fsencode(str(path)), C.addressof(h), out.ctypes.data, out.size))
    return out.reshape(dims), tuple(float(h.bounds[i]) for i in range(6)), h.params
