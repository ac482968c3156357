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
