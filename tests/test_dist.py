"""CPU, world_size 2 over gloo: the pose-sharded fusion merged with one all-reduce
equals the single-rank fusion bit for bit (the CPU oracle stands in for the GPU
kernel, which is exercised by the -m gpu tests and bench.py)."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _fuse(oracle, K, depth, poses, n):
    v = oracle.Volume()
    v.setDimensions(-0.5, 0.5, -0.5, 0.5, -0.5, 0.5)
    v.setVolumeSize(n, n, n)
    v.constructVolume()
    h, m, st = oracle.fuse_depth(v, K, depth, poses, dmin=200, dmax=1000)
    return h, m, st


def _worker(rank, world, port, K, depth, poses, n, out_dir):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "depth-map-fusion-utils_amd")]
    import torch
    import torch.distributed as dist
    from dmf_amd import dist as D
    from oracle import oracle
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    a, b = D.shard_range(len(poses), world, rank)
    h, m, st = _fuse(oracle, K, depth[a:b], poses[a:b], n)
    counters = torch.from_numpy(np.concatenate([h, m]))
    D.merge_counters(counters)
    tot = D.sum_over_ranks(st)
    t = D.max_over_ranks(float(rank + 1))
    np.save(os.path.join(out_dir, f"r{rank}.npy"), counters.numpy())
    np.save(os.path.join(out_dir, f"s{rank}.npy"), np.array(tot + [t]))
    dist.destroy_process_group()


@pytest.mark.parametrize("P,world", [(10, 2), (7, 3), (2, 2), (3, 8)])
def test_shard_range_partitions(P, world):
    from dmf_amd import dist as D
    seen = []
    for r in range(world):
        a, b = D.shard_range(P, world, r)
        seen += list(range(a, b))
    assert seen == list(range(P))


def test_sharded_fusion_gloo_world2(tmp_path, oracle):
    from dmf_amd import scene
    K = scene.K_640x480.copy()
    K[[0, 2, 4, 5]] *= np.float32(0.25)
    poses = scene.fibonacci_poses(5, seed=21)
    depth = scene.render_frames(K, 160, 120, poses)
    n = 48
    h, m, st = _fuse(oracle, K, depth, poses, n)
    mp.spawn(_worker, args=(2, _free_port(), K, depth, poses, n, str(tmp_path)), nprocs=2, join=True)
    for r in range(2):
        c = np.load(tmp_path / f"r{r}.npy")
        assert np.array_equal(c[: n ** 3], h) and np.array_equal(c[n ** 3:], m)
        s = np.load(tmp_path / f"s{r}.npy")
        assert np.array_equal(s[:3], st.astype(np.float64)) and s[3] == 2.0


def _vis_worker(rank, world, port, out_dir):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "depth-map-fusion-utils_amd"), os.path.join(root, "tests")]
    import torch
    import torch.distributed as dist
    import helpers as Hh
    from dmf_amd import dist as D
    from oracle import oracle
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    ov = Hh.oracle_volume(oracle, n=64)
    eng = oracle.Engine(Hh.K)
    poses = Hh.all_poses()

    def compute(block):
        res = [eng.reverseRayTraceFast(ov, T, True) for T in block]
        return [f for f, _ in res], [g for _, g in res]
    found, lists = D.sharded_visibility(compute, poses, world, rank)
    view, good, _, _ = ov.voxel_table()
    flags = torch.from_numpy(np.stack([view.astype(np.int32), good.astype(np.int32)]))
    D.merge_flags_max(flags)
    sel = oracle.greedy_set_cover(lists, 5)
    np.save(os.path.join(out_dir, f"v{rank}.npy"),
            np.array([len(x) for x in lists] + [int(f) for f in found] + list(sel), np.int64))
    np.save(os.path.join(out_dir, f"f{rank}.npy"), flags.numpy())
    dist.destroy_process_group()


def test_sharded_visibility_gloo_world2(tmp_path, oracle):
    """Pose-sharded reverseRayTraceFast (viz) over 2 gloo ranks: gathered lists, MAX-merged
    flags and the set cover on the gathered lists equal the single-rank run."""
    import helpers as Hh
    ov = Hh.oracle_volume(oracle, n=64)
    eng = oracle.Engine(Hh.K)
    poses = Hh.all_poses()
    res = [eng.reverseRayTraceFast(ov, T, True) for T in poses]
    lists = [g for _, g in res]
    view, good, _, _ = ov.voxel_table()
    exp = np.array([len(x) for x in lists] + [int(f) for f, _ in res] + list(oracle.greedy_set_cover(lists, 5)),
                   np.int64)
    mp.spawn(_vis_worker, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True)
    for r in range(2):
        assert np.array_equal(np.load(tmp_path / f"v{r}.npy"), exp)
        f = np.load(tmp_path / f"f{r}.npy")
        assert np.array_equal(f[0], view.astype(np.int32)) and np.array_equal(f[1], good.astype(np.int32))
