"""Multi-GPU pose sharding: poses are independent given the grid, so
P poses go to G ranks in contiguous blocks of ceil(P/G); every rank fuses its block
into its own replica of the int32 [hits | misses] counters and ONE all-reduce(SUM)
merges them (RCCL over xGMI with backend "nccl"; gloo on CPU).  Counts are exact
integers, so the merge is associative and bit-identical to a single-rank fusion.
The clamped int16 log-odds are finalized after the merge on every rank.
"""
from __future__ import annotations


def shard_range(P_total: int, world: int, rank: int):
    """[start, stop) of rank's contiguous pose block (ceil(P/G) per rank)."""
    per = -(-P_total // world)
    start = min(rank * per, P_total)
    return start, min(start + per, P_total)


def merge_counters(counters, group=None):
    """All-reduce(SUM) of the packed [hits | misses] int32 counters, in place."""
    import torch.distributed as dist
    if dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1:
        dist.all_reduce(counters, op=dist.ReduceOp.SUM, group=group)
    return counters


def max_over_ranks(value: float, device=None) -> float:
    """Max of a per-rank scalar (the bench's step time)."""
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return float(value)
    t = torch.tensor([float(value)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def sum_over_ranks(values, device=None):
    import torch
    import torch.distributed as dist
    t = torch.tensor([float(v) for v in values], dtype=torch.float64, device=device)
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return [float(x) for x in t.cpu().tolist()]


# ---- visibility queries (reverseRayTraceFast / set cover), SURVEY.md §8e ----------
# Queries only read the grid: rank r evaluates its contiguous pose block, the per-pose
# outputs are gathered in pose order (no data-path collective during the compute); the
# good flags merge with an all-reduce(MAX), the view ids with a min over non-zero ids.

def gather_pose_lists(found, lists, group=None):
    """All ranks' (found[], lists[]) of their pose blocks -> the full pose-ordered
    (found, lists) on every rank (all_gather_object; shards are contiguous)."""
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size(group) == 1:
        return list(found), list(lists)
    parts = [None] * dist.get_world_size(group)
    dist.all_gather_object(parts, (list(found), [list(map(int, x)) for x in lists]), group=group)
    f_all, l_all = [], []
    for f, l in parts:
        f_all += f
        l_all += l
    return f_all, l_all


def merge_flags_max(flags, group=None):
    """All-reduce(MAX) of a per-voxel flag tensor (good uint8 widened), in place."""
    import torch.distributed as dist
    if dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1:
        dist.all_reduce(flags, op=dist.ReduceOp.MAX, group=group)
    return flags


def merge_view_ids(view, group=None):
    """Voxel::view across pose shards, in place: the smallest non-zero id (0 = never viewed),
    as dmf_flags_allreduce (classify sets view only while it is 0, RayTracingEngine.hpp:354,
    so one rank walking the poses in order keeps the first pose's id)."""
    import torch
    import torch.distributed as dist
    if dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1:
        big = torch.iinfo(view.dtype).max
        view[view == 0] = big
        dist.all_reduce(view, op=dist.ReduceOp.MIN, group=group)
        view[view == big] = 0
    return view


def sharded_visibility(compute, poses, world, rank, group=None):
    """compute(pose_block) -> (found[], lists[]) on this rank's block (e.g.
    RayTracingEngine.reverseRayTraceFastBatch bound to a volume); returns the full
    pose-ordered results on every rank."""
    a, b = shard_range(len(poses), world, rank)
    found, lists = compute(poses[a:b]) if b > a else ([], [])
    return gather_pose_lists(found, lists, group)


# ---- merge + finalize (reduce-scatter / slab finalize / all-gather), DESIGN.md §7 ------
# The fusion counters are tiled (2x2x4-cell tiles of 16 int32, tiles x-major; DESIGN.md
# §6), so a contiguous range of whole tile rows (tx) is an x slab of the grid.  The
# counter arrays are padded to world * rows_per_rank tile rows; rank r reduces and
# finalizes rows [r*rows, (r+1)*rows) and the int16 slabs are all-gathered.  This moves
# 2*4 B (hits, misses) + 2 B (log-odds) per cell instead of the all-reduce's 2*2*4 B.
# The GPU path is libdmf's dmf_fuse_merge_finalize_device over an RCCL communicator; the
# gloo path below runs the same partition (libdmf's host-only dmf_fuse_merge_plan_dims)
# with torch collectives for CPU tests.

def tile_rows(dims):
    """(ntx, tiles per row) of the tiled counter layout of a grid (nx, ny, nz)."""
    nx, ny, nz = dims
    return (nx + 1) // 2, ((ny + 1) // 2) * ((nz + 3) // 4)


def rows_per_rank(dims, world):
    ntx, _ = tile_rows(dims)
    return -(-ntx // world)


def padded_counter_cells(dims, world):
    """= dmf_fuse_counter_cells_padded: elements per tiled counter array."""
    _, tpr = tile_rows(dims)
    return rows_per_rank(dims, world) * world * tpr * 16


def padded_logodds_cells(dims, world):
    """= dmf_fuse_logodds_cells_padded."""
    return rows_per_rank(dims, world) * world * 2 * dims[1] * dims[2]


def to_tiled(lin, dims, n_pad):
    """x-major int32 counters -> the tiled layout, zero-padded to n_pad elements."""
    import numpy as np
    nx, ny, nz = dims
    px, py, pz = -(-nx // 2) * 2, -(-ny // 2) * 2, -(-nz // 4) * 4
    g = np.zeros((px, py, pz), np.int32)
    g[:nx, :ny, :nz] = np.asarray(lin, np.int32).reshape(nx, ny, nz)
    # (tx, xi, ty, yi, tz, zi) -> (tx, ty, tz, xi, yi, zi)
    t = g.reshape(px // 2, 2, py // 2, 2, pz // 4, 4).transpose(0, 2, 4, 1, 3, 5).reshape(-1)
    out = np.zeros(n_pad, np.int32)
    out[: t.size] = t
    return out


def finalize_tiles_np(hits_t, miss_t, dims, l_hit, l_miss, l_min, l_max, out, t0, t1):
    """k_finalize over tiles [t0, t1) in numpy: writes out[x, y, z] (x-major int16)."""
    import numpy as np
    nx, ny, nz = dims
    nty, ntz = (ny + 1) // 2, (nz + 3) // 4
    for t in range(t0, t1):
        tz, r = t % ntz, t // ntz
        ty, tx = r % nty, r // nty
        h = hits_t[16 * t: 16 * t + 16].astype(np.int64).reshape(2, 2, 4)
        m = miss_t[16 * t: 16 * t + 16].astype(np.int64).reshape(2, 2, 4)
        L = np.clip(h * l_hit + m * l_miss, l_min, l_max).astype(np.int16)
        for xi in range(2):
            for yi in range(2):
                x, y = 2 * tx + xi, 2 * ty + yi
                if x < nx and y < ny:
                    z0 = 4 * tz
                    k = min(4, nz - z0)
                    out[(x * ny + y) * nz + z0: (x * ny + y) * nz + z0 + k] = L[xi, yi, :k]


def merge_finalize_gloo(counters, dims, prm, logodds, group=None):
    """dmf_fuse_merge_finalize_device over a torch.distributed group (gloo on CPU): the
    offsets and slab bounds come from libdmf's own plan (dmf_fuse_merge_plan_dims, the
    arithmetic the RCCL merge runs), the collectives from torch, the slab finalize from the
    numpy restatement of k_finalize.  counters = torch int32 [hits | misses] tiled, each
    plan["n_padded"]; logodds = torch int16 of plan["logodds_padded"], filled on every rank."""
    import torch
    import torch.distributed as dist
    from . import _lib
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    rank = dist.get_rank(group) if dist.is_initialized() else 0
    p = _lib.merge_plan_dims(dims, world, rank)
    n_pad, chunk, off = p["n_padded"], p["chunk"], p["chunk_offset"]
    hits, miss = counters[:n_pad], counters[n_pad: 2 * n_pad]
    for arr in (hits, miss):
        part = torch.empty(chunk, dtype=torch.int32)
        if world > 1:
            dist.reduce_scatter_tensor(part, arr, group=group)
        else:
            part.copy_(arr[:chunk])
        arr[off: off + chunk] = part
    out = logodds.numpy()
    finalize_tiles_np(hits.numpy(), miss.numpy(), dims, prm["l_hit"], prm["l_miss"], prm["l_min"], prm["l_max"],
                      out, p["tile_begin"], p["tile_end"])
    if world > 1:
        sb, so = p["slab_bytes"] // 2, p["slab_offset"] // 2  # int16 elements
        mine = logodds[so: so + sb].clone().view(torch.uint8)
        allb = torch.empty(world * sb * 2, dtype=torch.uint8)
        dist.all_gather_into_tensor(allb, mine, group=group)
        logodds.copy_(allb.view(torch.int16))
    return logodds


def merge_finalize_device(vol, counters, prm_ptr, logodds, comm_ptr, stream_ptr=None):
    """GPU: libdmf's dmf_fuse_merge_finalize_device over an RCCL communicator (e.g. torch's
    ProcessGroupNCCL._comm_ptr(); None = a single rank: the finalize alone) on stream_ptr (None = the
    volume's stream)."""
    from . import _lib
    _lib.check(vol._L.dmf_fuse_merge_finalize_device(vol._h, counters.data_ptr(), prm_ptr, logodds.data_ptr(),
                                                     comm_ptr, stream_ptr))


def torch_comm_ptr(group=None, device=None):
    """ncclComm_t of torch's NCCL(=RCCL) process group, as an int (connects it eagerly)."""
    import torch
    import torch.distributed as dist
    pg = group or dist.distributed_c10d._get_default_group()
    be = pg._get_backend(device or torch.device("cuda", torch.cuda.current_device()))
    ptr = int(be._comm_ptr())
    if ptr == 0:
        raise RuntimeError("RCCL communicator not initialised (run a collective or eager_connect first)")
    return ptr
