"""CPU, world_size 2 over gloo: the pose-sharded fusion merged with one all-reduce
equals the single-rank fusion bit for bit (the CPU oracle stands in for the GPU
kernel, which is exercised by the -m gpu tests and bench.py)."""
import json
import os
import socket
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp


ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


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
    v_ids = torch.from_numpy(view.astype(np.int32))
    D.merge_view_ids(v_ids)
    g_fl = torch.from_numpy(good.astype(np.int32))
    D.merge_flags_max(g_fl)
    flags = torch.stack([v_ids, g_fl])
    sel = oracle.greedy_set_cover(lists, 5)
    np.save(os.path.join(out_dir, f"v{rank}.npy"),
            np.array([len(x) for x in lists] + [int(f) for f in found] + list(sel), np.int64))
    np.save(os.path.join(out_dir, f"f{rank}.npy"), flags.numpy())
    dist.destroy_process_group()


def test_sharded_visibility_gloo_world2(tmp_path, oracle):
    """Pose-sharded reverseRayTraceFast (viz) over 2 gloo ranks: gathered lists, merged
    flags (good: max, view: min non-zero id) and the set cover on the gathered lists equal
    the single-rank run."""
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


# ---- the bench's step schedule (dmf_amd.schedule.run_steps) over 2 gloo ranks -------
# Each rank runs the real schedule on the randomized stream simulator: fuse = the CPU
# oracle into tiled counters, merge = the reduce-scatter / slab finalize / all-gather
# restatement of dmf_fuse_merge_finalize_device.  Step i fuses frames {i, i+S} (one per
# rank), so every step's merged log-odds differ and buffer mix-ups show.

def _sched_worker(rank, world, port, K, depth, poses, n, nsteps, seeds, reuse_wait, out_dir, phase=False):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "depth-map-fusion-utils_amd")]
    import torch
    import torch.distributed as dist
    from dmf_amd import dist as D
    from dmf_amd import schedule as S
    from oracle import oracle
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    dims = (n, n, n)
    prm = {"l_hit": 847, "l_miss": -405, "l_min": -2000, "l_max": 3511}
    npad = D.padded_counter_cells(dims, world)
    results = []
    for seed in seeds:
        bufs = [torch.zeros(2 * npad, dtype=torch.int32) for _ in range(2)]
        logodds = torch.zeros(D.padded_logodds_cells(dims, world), dtype=torch.int16)
        out = {}

        def clear(b):
            bufs[b].zero_()

        def fuse(b, i):
            f = i + rank * nsteps  # this rank's frame of step i
            h, m, _ = _fuse(oracle, K, depth[f:f + 1], poses[f:f + 1], n)
            bufs[b][:npad] += torch.from_numpy(D.to_tiled(h, dims, npad))
            bufs[b][npad:] += torch.from_numpy(D.to_tiled(m, dims, npad))

        def merge(b, i):
            D.merge_finalize_gloo(bufs[b], dims, prm, logodds)
            out[i] = logodds[: n ** 3].clone().numpy()

        rt = S.SimRuntime(seed)
        # phase: step i-1's merge also waits for an event recorded on compute after step i's
        # fusion (the simulator's stand-in for the phase-F event of dmf_fuse_set_phase_event)
        S.run_steps(rt, nsteps, 2, clear, fuse, merge, reuse_wait=reuse_wait,
                    phase=(lambda i: rt.record("compute")) if phase else None)
        results.append(np.stack([out[i] for i in range(nsteps)]))
    np.save(os.path.join(out_dir, f"sched{rank}.npy"), np.stack(results))
    dist.destroy_process_group()


def _sched_expected(oracle, K, depth, poses, n, nsteps):
    exp = []
    for i in range(nsteps):
        idx = [i, i + nsteps]
        h, m, _ = _fuse(oracle, K, depth[idx], poses[idx], n)
        L = np.clip(h.astype(np.int64) * 847 + m.astype(np.int64) * -405, -2000, 3511).astype(np.int16)
        exp.append(L)
    return np.stack(exp)


def _sched_inputs():
    from dmf_amd import scene
    K = scene.K_640x480.copy()
    K[[0, 2, 4, 5]] *= np.float32(0.125)
    nsteps = 3
    poses = scene.fibonacci_poses(2 * nsteps, seed=5)
    depth = scene.render_frames(K, 80, 60, poses)
    return K, depth, poses, nsteps


@pytest.mark.parametrize("phase", [False, True])
def test_step_schedule_gloo_world2(tmp_path, oracle, phase):
    """The pipelined schedule (merge of step i overlapping fuse of step i+1, two counter
    buffers; phase: the merge of step i deferred behind step i+1's phase-F event, as the bench
    runs it) on 2 ranks under random stream-consistent execution orders: every step's
    merged, finalized log-odds equal the single-rank fusion of that step's frames."""
    K, depth, poses, nsteps = _sched_inputs()
    n = 21  # odd: a partial last tile row, and 11 tile rows over 2 ranks (padding)
    exp = _sched_expected(oracle, K, depth, poses, n, nsteps)
    seeds = [1, 2, 3, 4]
    mp.spawn(_sched_worker, args=(2, _free_port(), K, depth, poses, n, nsteps, seeds, True, str(tmp_path), phase),
             nprocs=2, join=True)
    for r in range(2):
        got = np.load(tmp_path / f"sched{r}.npy")
        for s in range(len(seeds)):
            assert np.array_equal(got[s], exp), (r, s)


def test_step_schedule_needs_reuse_wait(tmp_path, oracle):
    """Negative control: without the wait for a buffer's previous merge before it is
    cleared, some random execution order corrupts a step (the simulator can see it)."""
    K, depth, poses, nsteps = _sched_inputs()
    n = 16
    exp = _sched_expected(oracle, K, depth, poses, n, nsteps)
    seeds = list(range(10, 22))
    mp.spawn(_sched_worker, args=(2, _free_port(), K, depth, poses, n, nsteps, seeds, False, str(tmp_path)),
             nprocs=2, join=True)
    bad = 0
    for r in range(2):
        got = np.load(tmp_path / f"sched{r}.npy")
        bad += sum(not np.array_equal(got[s], exp) for s in range(len(seeds)))
    assert bad > 0


@pytest.mark.parametrize("dims", [(5, 3, 6), (21, 21, 21), (61, 61, 61), (1024, 1024, 288), (7, 1, 1)])
@pytest.mark.parametrize("world", [1, 2, 3, 8])
def test_merge_plan_partitions_the_grid(dims, world):
    """libdmf's merge plan (the slab arithmetic of the RCCL merge, dmf_fuse_merge_plan_dims)
    against the padded sizes restated here: the ranks' reduce-scatter chunks tile the padded
    counter arrays, their finalize tile ranges tile the grid's tiles in rank order, and
    their log-odds slabs tile the padded int16 grid."""
    from dmf_amd import _lib
    from dmf_amd import dist as D
    ntx, tpr = D.tile_rows(dims)
    whole = _lib.merge_plan_dims(dims, world, -1)
    assert whole["tile_begin"] == 0 and whole["tile_end"] == ntx * tpr
    t = 0
    for r in range(world):
        p = _lib.merge_plan_dims(dims, world, r)
        assert p["n_padded"] == D.padded_counter_cells(dims, world) == whole["n_padded"]
        assert p["logodds_padded"] == D.padded_logodds_cells(dims, world)
        assert p["chunk"] * world == p["n_padded"] and p["chunk_offset"] == r * p["chunk"]
        assert p["slab_bytes"] * world == 2 * p["logodds_padded"] and p["slab_offset"] == r * p["slab_bytes"]
        assert p["tile_begin"] == t and p["tile_end"] >= p["tile_begin"]
        # a rank's tiles lie inside its own reduce-scatter chunk and its own log-odds slab
        # (ranks past the grid's last tile row hold padding only: an empty range)
        if p["tile_end"] > p["tile_begin"]:
            assert p["chunk_offset"] <= 16 * p["tile_begin"] and 16 * p["tile_end"] <= p["chunk_offset"] + p["chunk"]
            x0 = 2 * (p["tile_begin"] // tpr)
            x1 = min(dims[0], 2 * (p["tile_end"] // tpr))
            lo = 2 * x0 * dims[1] * dims[2]
            assert p["slab_offset"] <= lo and 2 * x1 * dims[1] * dims[2] <= p["slab_offset"] + p["slab_bytes"]
        t = p["tile_end"]
    assert t == ntx * tpr


def test_merge_partition_single_rank():
    """Padded sizes and the tiled slab finalize (numpy restatement) at world 1 and 3."""
    from dmf_amd import dist as D
    for dims in [(5, 3, 6), (21, 21, 21), (8, 2, 4)]:
        lin_h = np.random.default_rng(0).integers(0, 9, size=np.prod(dims)).astype(np.int32)
        lin_m = np.random.default_rng(1).integers(0, 9, size=np.prod(dims)).astype(np.int32)
        exp = np.clip(lin_h.astype(np.int64) * 847 + lin_m * -405, -2000, 3511).astype(np.int16)
        for world in (1, 3):
            npad = D.padded_counter_cells(dims, world)
            ht, mt = D.to_tiled(lin_h, dims, npad), D.to_tiled(lin_m, dims, npad)
            out = np.zeros(D.padded_logodds_cells(dims, world), np.int16)
            ntx, tpr = D.tile_rows(dims)
            rows = D.rows_per_rank(dims, world)
            for r in range(world):  # every rank's slab, as the all-gather assembles them
                r0, r1 = min(ntx, r * rows), min(ntx, (r + 1) * rows)
                D.finalize_tiles_np(ht, mt, dims, 847, -405, -2000, 3511, out, r0 * tpr, r1 * tpr)
            assert np.array_equal(out[: exp.size], exp)
            assert npad >= ((dims[0] + 1) // 2) * tpr * 16


def _bench(*args, env_extra=None):
    import subprocess
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], stdout=subprocess.PIPE,
                          stderr=subprocess.PIPE, env=env, timeout=300, text=True)


@pytest.mark.parametrize("n", [2, 8])
def test_bench_spawns_its_ranks(n):
    """`python bench.py --gpus N` (N > 1, no launcher) starts N ranks itself: a
    torch.distributed.run child with one rank per GPU on 127.0.0.1, every argument forwarded
    (--print-launch is the dry run: it prints the command and touches no GPU)."""
    r = _bench("--gpus", str(n), "--steps", "7", "--warmup", "3", "--print-launch")
    assert r.returncode == 0, r.stderr
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1
    cmd = json.loads(lines[0])["launch"]
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nnodes=1" in cmd and f"--nproc-per-node={n}" in cmd
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert int(cmd[cmd.index("--master-port") + 1]) > 0
    i = cmd.index(os.path.join(ROOT, "bench.py"))
    assert cmd[i + 1:] == ["--gpus", str(n), "--steps", "7", "--warmup", "3"]


def test_bench_rejects_world_mismatch():
    """A launcher whose WORLD_SIZE differs from --gpus is an error, not a warning."""
    r = _bench("--gpus", "4", "--steps", "1", env_extra={"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode != 0
    assert "WORLD_SIZE=2" in r.stderr
