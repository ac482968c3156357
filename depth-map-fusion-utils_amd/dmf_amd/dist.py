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
# outputs are gathered in pose order (no data-path collective during the compute), and
# the idempotent view/good flags merge with an all-reduce(MAX).

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
    """All-reduce(MAX) of a per-voxel flag tensor (view int32 / good uint8 widened), in place."""
    import torch.distributed as dist
    if dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1:
        dist.all_reduce(flags, op=dist.ReduceOp.MAX, group=group)
    return flags


def sharded_visibility(compute, poses, world, rank, group=None):
    """compute(pose_block) -> (found[], lists[]) on this rank's block (e.g.
    RayTracingEngine.reverseRayTraceFastBatch bound to a volume); returns the full
    pose-ordered results on every rank."""
    a, b = shard_range(len(poses), world, rank)
    found, lists = compute(poses[a:b]) if b > a else ([], [])
    return gather_pose_lists(found, lists, group)
