#!/usr/bin/env python3
"""Headline benchmark: ray-voxel updates/s of the 3D-DDA log-odds depth fusion step
(BASELINE.json metric "ray-voxel updates/sec + Mrays/sec, 512^3 grid, 640x480 depth
@ 1/2/4/8 GPU"; workload = config 4 sharded: 128 poses of 640x480 depth per GPU
into a replicated 512^3 grid, N=8 -> 1024 poses).

One step = clear the int32 hit/miss counters, fuse the rank's 128 depth frames
(back-projection + exact integer 3D-DDA, libdmf.so brick pipeline k_bk_*), merge the
ranks' counters (N>1: RCCL reduce-scatter, slab finalize, all-gather of the int16 slabs,
libdmf dmf_fuse_merge_finalize_device) or finalize (N=1) to the clamped int16 log-odds
grid.  The merge of step i and the clear of its buffer overlap the fusion of step i+1
(dmf_amd.schedule).  Inputs
are resident in HBM before timing starts.

Launch: python bench.py [--gpus N --steps K --warmup W]; for N>1 through
torch.distributed.run (one rank per GPU, RCCL over xGMI).  Rank 0 prints ONE JSON line.
"""
from __future__ import annotations

import argparse
import csv
import datetime
import ctypes as C
import glob
import hashlib
import json
import os
import shutil
import subprocess
import sys
import tempfile
import time

import numpy as np
import torch  # import before libdmf.so: both must share torch's HIP runtime
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, "depth-map-fusion-utils_amd")
sys.path[:0] = [ROOT, PKG]

import dmf_amd  # noqa: E402
from dmf_amd import _lib, scene  # noqa: E402
from dmf_amd import dist as D  # noqa: E402
from dmf_amd import schedule as S  # noqa: E402

GRID = 512
WIDTH, HEIGHT = 640, 480
POSES_PER_GPU = 128
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
# VALU issue peak: 256 CUs x 4 SIMD-32 x one wave64 VALU instruction per 2 cycles at 2.4 GHz
# (MI355X_MICROARCH.md "Wave scheduling"), in wave-instructions/s
VALU_PEAK_WIPS = 256 * 4 * 2.4e9 / 2
# LDS-add peak: 256 CUs x one ds_add_u32 wave-instruction per 4 cycles (address + data moved to
# the LDS at 2 cycles per dword per wave-instruction, MI355X_MICROARCH.md §LDS) at 2.4 GHz
LDS_ADD_PEAK_WIPS = 256 * 2.4e9 / 4
BYTES_PER_UPDATE = 4   # int16 read + int16 write per cell update
BYTES_PER_DEPTH = 2    # uint16 depth read per pixel


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def make_inputs(rank, world, P_local, cache_dir="/tmp/dmf_bench_cache"):
    """Rank's shard of a Fibonacci pose sphere (P_local*world poses) + rendered depth."""
    P_total = P_local * world
    a, b = D.shard_range(P_total, world, rank)
    poses = scene.fibonacci_poses(P_total, seed=1234)[a:b]
    os.makedirs(cache_dir, exist_ok=True)
    key = os.path.join(cache_dir, f"depth_{WIDTH}x{HEIGHT}_P{P_total}_r{rank}_of{world}.npy")
    if os.path.exists(key):
        depth = np.load(key)
    else:
        depth = scene.render_frames(scene.intrinsics(WIDTH, HEIGHT), WIDTH, HEIGHT, poses)
        np.save(key, depth)
    return poses, depth


def workload_name(grid, P, world):
    """Which BASELINE.json config the run reproduces (per-GPU shard for the 8-GPU ones)."""
    if (WIDTH, HEIGHT, grid) == (640, 480, 256) and P * world == 64:
        return "config2"
    if (WIDTH, HEIGHT, grid) == (1280, 720, 512) and P * world == 256:
        return "config3"
    if (WIDTH, HEIGHT, grid) == (1280, 720, 1024) and P == 256:
        return "config5-shard (2048 poses / 8 GPUs)"
    if (WIDTH, HEIGHT, grid) == (1280, 720, 1024):
        return "config5-grid (fewer poses than its 256-pose shard)"
    if (WIDTH, HEIGHT, grid) == (640, 480, 512) and P * world == 1024 and world == 1:
        return "config4-anchor (all 1024 poses on one GPU)"
    if (WIDTH, HEIGHT, grid) == (640, 480, 512):
        return "config4-shard"
    return "custom"


def cpu_baseline(K, poses, depth, n_frames, grid, threads=1):
    """Oracle (CPU restatement; threads > 1 = its OpenMP row-parallel variant) on a
    bounded sample of the same workload."""
    from oracle import oracle as O
    v = O.Volume()
    v.setDimensions(-0.5, 0.5, -0.5, 0.5, -0.5, 0.5)
    v.setVolumeSize(grid, grid, grid)
    v.constructVolume()
    n = grid ** 3
    hits = np.zeros(n, np.int32)
    misses = np.zeros(n, np.int32)
    t0 = time.perf_counter()
    _, _, st = O.fuse_depth(v, K, depth[:n_frames], poses[:n_frames], dmin=scene.DEPTH_MIN_MM,
                            dmax=scene.DEPTH_MAX_MM, hits=hits, misses=misses, threads=threads)
    dt = time.perf_counter() - t0
    return float(st[0]) / dt, float(st[1]) / dt, dt


def reference_fusion_baseline(K, poses, depth, n_frames, grid, budget_s=20.0):
    """The reference's OWN fusion path on the host, timed on the same frames: per frame the
    oracle's Camera::projectPoint + transformPoints back-projection (Camera.hpp:24-45, the
    cloud a reference driver integrates) and VoxelVolume::integratePointCloud(cloud, normals)
    (Volume.hpp:199-228) in the reference layout -- vector<vector<vector<Voxel*>>>, one `new
    Voxel` per first touch, push_back of every point and normal -- single-threaded, as the
    reference is.  The reference integrates each point into ONE voxel (no ray traversal), so
    its ray-voxel updates are its points.  Frames run until `budget_s` is spent (at most
    n_frames).  Normals are unit vectors (their values do not change the work)."""
    from oracle import oracle as O
    v = O.Volume()
    v.setDimensions(-0.5, 0.5, -0.5, 0.5, -0.5, 0.5)
    v.setVolumeSize(grid, grid, grid)
    v.constructVolume()
    t_bp = t_int = 0.0
    npts = nfr = 0
    for i in range(n_frames):
        t0 = time.perf_counter()
        xyz = O.backproject(K, depth[i], poses[i])
        m = depth[i] > 0
        pts = np.ascontiguousarray(xyz[m])
        t1 = time.perf_counter()
        nrm = np.zeros_like(pts)
        nrm[:, 2] = 1.0
        t2 = time.perf_counter()
        v.integratePointCloud(pts, nrm)
        t3 = time.perf_counter()
        t_bp += t1 - t0
        t_int += t3 - t2
        npts += int(pts.shape[0])
        nfr += 1
        if t_bp + t_int > budget_s:
            break
    return {"value": npts / (t_bp + t_int), "unit": "ray-voxel updates/s (= points/s: one voxel per point)",
            "cores": 1, "kind": "port",
            "integrate_points_per_s": npts / t_int, "backproject_points_per_s": npts / t_bp,
            "occupied_voxels": len(v.occupied_cells_),
            "sample": f"oracle reference-layout back-projection + integratePointCloud(cloud, normals) of {nfr} of the "
                      f"{len(poses)} frames ({npts} points, {grid}^3), {t_bp + t_int:.1f}s single-threaded "
                      f"(integrate {t_int:.1f}s, back-projection {t_bp:.1f}s); the reference's own fusion, "
                      "Volume.hpp:199-228"}


# PMC passes of the live measurement (one rocprofv3 run each; FETCH_SIZE takes 3 of the 4
# TCC slots and WRITE_SIZE 2, so they cannot share a pass: MI355X_MICROARCH.md §PMC slots)
PMC_PASSES = (["FETCH_SIZE"], ["WRITE_SIZE"],
              ["SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_WAVE_CYCLES", "SQ_BUSY_CYCLES",
               "SQ_LDS_BANK_CONFLICT", "TCC_HIT_sum", "TCC_MISS_sum"])


def pmc_measure(args, log_dir=None):
    """HBM traffic and instruction counts of THIS configuration, measured now: the same
    workload (one step, one fusion call, the secondary kernels) re-run as a child process
    under `rocprofv3 --pmc`, one pass per counter group.  Returns {kernel: {counter:
    (total, dispatches)}} or None when rocprofv3 is unavailable or a pass fails (the bench
    line then reports traffic null).  Traffic is corrected as MI355X_MICROARCH.md
    prescribes for gfx950: bytes = (2 x FETCH_SIZE + WRITE_SIZE) x 1024."""
    prof = shutil.which("rocprofv3")
    if prof is None or under_profiler():
        return None
    tmp = tempfile.mkdtemp(prefix="dmf_pmc_", dir=os.environ.get("TMPDIR", "/tmp"))
    child = [sys.executable, os.path.abspath(__file__), "--pmc", "off", "--steps", "1", "--warmup", "0",
             "--cpu-frames", "0", "--grid", str(args.grid), "--poses-per-gpu", str(args.poses_per_gpu),
             "--image", args.image, "--serial-ref", "off", "--cpu-reverse-poses", "0"] + (
                 ["--no-secondary"] if args.no_secondary else [])
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK")}
    env.setdefault("TMPDIR", "/tmp")
    out = {}
    try:
        for i, counters in enumerate(PMC_PASSES):
            d = os.path.join(tmp, f"p{i}")
            cmd = [prof, "--pmc", *counters, "--output-format", "csv", "-d", d, "-o", "run", "--"] + child
            r = subprocess.run(cmd, stdout=subprocess.DEVNULL, stderr=subprocess.PIPE, env=env, timeout=300)
            if r.returncode != 0:
                log(f"pmc pass {counters} failed ({r.returncode}): {r.stderr.decode(errors='replace')[-400:]}")
                return None
            files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
            if not files:
                return None
            for f in files:
                for row in csv.DictReader(open(f)):
                    k = row["Kernel_Name"].split("(")[0].replace("void ", "").strip()
                    if not k.startswith("dmf::"):
                        continue
                    e = out.setdefault(k, {}).setdefault(row["Counter_Name"], [0.0, set()])
                    e[0] += float(row["Counter_Value"])
                    e[1].add(row["Dispatch_Id"])
        # kernel durations of the same workload in its timed mode (a short pipelined run): the
        # per-kernel averages beside the step interval, F's among them
        d = os.path.join(tmp, "kt")
        kt_child = [c if c != "1" or child[i - 1] != "--steps" else "20" for i, c in enumerate(child)]
        cmd = [prof, "--kernel-trace", "--stats", "--output-format", "csv", "-d", d, "-o", "run", "--"] + kt_child
        r = subprocess.run(cmd, stdout=subprocess.DEVNULL, stderr=subprocess.PIPE, env=env, timeout=300)
        kt = {}
        if r.returncode == 0:
            for f in glob.glob(os.path.join(d, "**", "*kernel_stats.csv"), recursive=True):
                for row in csv.DictReader(open(f)):
                    k = row["Name"].split("(")[0].replace("void ", "").strip()
                    if k.startswith("dmf::"):
                        kt[k] = {"avg_ms": float(row["AverageNs"]) * 1e-6, "calls": int(row["Calls"])}
        else:
            log(f"kernel-trace pass failed ({r.returncode}): {r.stderr.decode(errors='replace')[-400:]}")
        if log_dir:
            shutil.copytree(tmp, log_dir, dirs_exist_ok=True)
    except (OSError, subprocess.SubprocessError, ValueError, KeyError) as ex:
        log(f"pmc measurement skipped: {ex}")
        return None
    finally:
        shutil.rmtree(tmp, ignore_errors=True)
    res = {k: {c: (v[0], len(v[1])) for c, v in cs.items()} for k, cs in out.items()}
    res["__kernel_trace__"] = kt
    return res


def under_profiler():
    """True when this process already runs under rocprofv3 (its tool library is preloaded and
    it exports ROCPROF* settings): no nested profiler runs then."""
    return "rocprof" in os.environ.get("LD_PRELOAD", "") or any(k.startswith("ROCPROF") for k in os.environ)


def pmc_total(pmc, kernels, counter):
    """Sum over the kernels of a counter's total (all dispatches of the child run)."""
    return sum(pmc.get(k, {}).get(counter, (0.0, 0))[0] for k in kernels)


def pmc_per_dispatch(pmc, kernel, counter):
    t, n = pmc.get(kernel, {}).get(counter, (0.0, 0))
    return t / n if n else None


def issue_roofline(pmc, kernel, ms):
    """Issue-bound pricing of a march kernel (its occupancy bitmask is L2-resident, so HBM
    bytes say nothing): VALU wave-instructions per launch / launch time vs the VALU issue
    peak, with the L2 hit rate beside it."""
    valu = pmc_per_dispatch(pmc, kernel, "SQ_INSTS_VALU") if pmc else None
    if not valu or not ms:
        return None
    hit = pmc_per_dispatch(pmc, kernel, "TCC_HIT_sum") or 0.0
    miss = pmc_per_dispatch(pmc, kernel, "TCC_MISS_sum") or 0.0
    ach = valu / (ms * 1e-3)
    return {"bound": "valu-issue", "achieved": ach, "peak": VALU_PEAK_WIPS, "unit": "wave-instr/s",
            "frac": ach / VALU_PEAK_WIPS, "kernel": kernel, "valu_per_launch": valu,
            "salu_per_launch": pmc_per_dispatch(pmc, kernel, "SQ_INSTS_SALU"),
            "l2_hit_rate": hit / (hit + miss) if hit + miss > 0 else None,
            "hbm_bytes_per_launch": 1024.0 * (2.0 * (pmc_per_dispatch(pmc, kernel, "FETCH_SIZE") or 0.0)
                                              + (pmc_per_dispatch(pmc, kernel, "WRITE_SIZE") or 0.0)),
            "basis": "rocprofv3 PMC of the same workload in a child run; peak = 1024 SIMD-32 x 1 wave64 VALU "
                     "instruction / 2 cycles x 2.4 GHz"}


def one_rccl_mapped():
    """libdmf's RCCL calls take torch's communicator pointer: both must be the same
    librccl instance (same soname, loaded once by torch).  True if exactly one is mapped."""
    try:
        maps = open("/proc/self/maps").read().splitlines()
    except OSError:
        return False
    paths = {ln.split()[-1] for ln in maps if "librccl" in ln}
    return len(paths) == 1


GOLDEN = os.path.join(ROOT, "tests", "golden", "fusion_digests.json")


def expected_digest(grid, P_total):
    """The oracle's log-odds digest of this run's GLOBAL pose set (fibonacci_poses(P_total,
    seed=1234), bench make_inputs) at full size, committed by tests/golden/gen_fusion_digests.py,
    or None when that workload was not generated."""
    try:
        table = json.load(open(GOLDEN))
    except (OSError, ValueError):
        return None
    for key, e in table.items():
        if (e["grid"], e["image"], e["global_poses"], e["seed"]) == (grid, f"{WIDTH}x{HEIGHT}", P_total, 1234):
            return dict(e, key=key)
    return None


def host_cores():
    """The GPU box host's CPUs as the OS reports them (nproc / lscpu), beside the threads the
    CPU baselines used (the job's share, host_threads)."""
    info = {"os_cpu_count": os.cpu_count(), "affinity": len(os.sched_getaffinity(0)),
            "physical_cores_in_affinity": physical_cores_in_affinity(), "cgroup_cpu_quota": cgroup_cpu_quota(),
            "omp_num_threads_env": os.environ.get("OMP_NUM_THREADS")}
    try:
        out = subprocess.run(["lscpu"], stdout=subprocess.PIPE, stderr=subprocess.DEVNULL, timeout=10,
                             text=True).stdout
        for ln in out.splitlines():
            k, _, v = ln.partition(":")
            if k.strip() in ("Model name", "Socket(s)", "Core(s) per socket", "Thread(s) per core", "CPU(s)"):
                info[k.strip()] = v.strip()
    except (OSError, subprocess.SubprocessError):
        pass
    return info


def cgroup_cpu_quota():
    """CPUs the job's cgroup may use (cpu.max quota / period), or None when unlimited."""
    for path in ("/sys/fs/cgroup/cpu.max",):
        try:
            q, p = open(path).read().split()[:2]
            if q != "max":
                return float(q) / float(p)
        except (OSError, ValueError):
            pass
    try:  # cgroup v1
        q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
        p = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
        if q > 0 and p > 0:
            return q / p
    except (OSError, ValueError):
        pass
    return None


def physical_cores_in_affinity():
    """Distinct physical cores (socket, core id) among the CPUs this process may run on."""
    cpus = sorted(os.sched_getaffinity(0))
    seen = set()
    for c in cpus:
        try:
            base = f"/sys/devices/system/cpu/cpu{c}/topology/"
            seen.add((open(base + "physical_package_id").read().strip(), open(base + "core_id").read().strip()))
        except OSError:
            seen.add(("?", str(c)))
    return len(seen)


def host_threads(requested=0):
    """Threads for the multi-core CPU baselines: the physical cores of the affinity mask (one
    thread per core), bounded by the job's CPU share where the host enforces one -- a cgroup
    quota, or OMP_NUM_THREADS (the GPU box exports its share there: 16 per GPU) -- since threads
    beyond the share only time-slice.  `requested` > 0 overrides.  Returns (threads, reason)."""
    if requested > 0:
        return requested, "--cpu-threads"
    cores = physical_cores_in_affinity()
    quota = cgroup_cpu_quota()
    omp = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    n, why = cores, f"physical cores in the affinity mask ({cores})"
    if quota is not None and int(quota) < n:
        n, why = max(1, int(quota)), f"cgroup cpu.max quota {quota:g} CPUs < {cores} physical cores"
    if omp > 0 and omp < n:
        n, why = omp, f"OMP_NUM_THREADS={omp} (the job's CPU share) < {cores} physical cores"
    return max(1, n), why


def free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


class MergeError(RuntimeError):
    """libdmf's merge (dmf_fuse_merge_finalize_device) failed: the only error the warmup's RCCL
    fallback takes."""


def launch_command(args, argv):
    """The torch.distributed.run command of `bench.py --gpus N` (N > 1, no WORLD_SIZE): one rank
    per GPU of this node, rendezvous on 127.0.0.1, every bench argument forwarded unchanged
    (--print-launch dropped)."""
    fwd = [a for a in argv if a != "--print-launch"]
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
            "--master-addr", "127.0.0.1", "--master-port", str(free_port()), os.path.abspath(__file__)] + fwd


def launch_ranks(args, json_fd):
    """Spawn the N ranks as a child process, relay rank 0's JSON line on the real stdout and
    return the child's exit status.  The child's stderr passes through (progress, RCCL)."""
    cmd = launch_command(args, sys.argv[1:])
    if args.print_launch:
        os.write(json_fd, (json.dumps({"launch": cmd}) + "\n").encode())
        return 0
    log(f"bench: starting {args.gpus} ranks: {' '.join(cmd)}")
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC only on this pool (RCCL)
    proc = subprocess.run(cmd, stdout=subprocess.PIPE, env=env)
    lines = [ln for ln in proc.stdout.decode(errors="replace").splitlines() if ln.strip()]
    out = [ln for ln in lines if ln.lstrip().startswith("{") and '"metric"' in ln]
    for ln in lines:
        if ln not in out:
            log(f"[ranks stdout] {ln}")
    if out:
        os.write(json_fd, (out[-1].strip() + "\n").encode())
    elif proc.returncode == 0:
        log("bench: the ranks exited 0 but rank 0 printed no JSON line")
        return 1
    return proc.returncode


def main():
    # stdout carries exactly ONE JSON line (rank 0): anything else written to fd 1 by the
    # native libraries (e.g. RCCL's init banner) is sent to stderr
    sys.stdout.flush()
    json_fd = os.dup(1)
    os.dup2(2, 1)
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=1000)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--grid", type=int, default=GRID)
    ap.add_argument("--poses-per-gpu", type=int, default=POSES_PER_GPU)
    ap.add_argument("--cpu-frames", type=int, default=8, help="frames in the CPU-oracle baseline sample (0=skip)")
    ap.add_argument("--no-secondary", action="store_true")
    ap.add_argument("--pmc", default="auto", choices=["auto", "off"],
                    help="auto: at N=1, measure HBM traffic and instruction counts of this workload with "
                         "rocprofv3 PMC passes (child runs) after the timed region")
    ap.add_argument("--pmc-dir", default=None, help="keep the rocprofv3 PMC output here")
    ap.add_argument("--serial-ref", default="on", choices=["on", "off"],
                    help="pipelined runs: re-time the serial fusion call after the timed region")
    ap.add_argument("--cpu-reverse-poses", type=int, default=16,
                    help="poses of the multi-core reverseRayTraceFast CPU sample (0 = skip both samples)")
    ap.add_argument("--image", default="640x480", choices=["640x480", "1280x720"],
                    help="depth frame size (BASELINE configs 1/2/4: 640x480; 3/5: 1280x720)")
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="threads of the multi-core CPU baselines (0 = the job's CPU share, host_threads())")
    ap.add_argument("--print-launch", action="store_true",
                    help="--gpus N > 1 without WORLD_SIZE: print the torch.distributed.run command the bench would "
                         "spawn (JSON) and exit")
    args = ap.parse_args()
    global WIDTH, HEIGHT
    WIDTH, HEIGHT = (int(v) for v in args.image.split("x"))

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # `python bench.py --gpus N` starts its own N ranks: torch.distributed.run as a CHILD
        # process (never exec: nothing here has touched the GPU yet, and nothing will in this
        # parent), whose rank 0 prints the JSON line; the parent relays it and exits with the
        # child's status
        sys.exit(launch_ranks(args, json_fd))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}: launch N ranks with --gpus N "
                         "(or run `python bench.py --gpus N` without a launcher: it starts the ranks itself)")
    # DMF_BENCH_BACKEND=gloo rehearses the N > 1 path with ranks sharing GPUs (no RCCL: the
    # merge falls back to torch's all-reduce + finalize); the driver's runs use nccl (= RCCL)
    backend = os.environ.get("DMF_BENCH_BACKEND", "nccl")
    local_rank = local_rank % max(torch.cuda.device_count(), 1)
    torch.cuda.set_device(local_rank)
    ctl_group = None
    if world > 1:
        # torch's collectives time out instead of hanging for ever
        tmo = datetime.timedelta(seconds=int(os.environ.get("DMF_BENCH_DIST_TIMEOUT_S", "600")))
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank), timeout=tmo)
        else:
            dist.init_process_group(backend, timeout=tmo)
        # a CPU group for the ranks' agreement on the merge path (it must work whatever state
        # the GPU communicator is in)
        ctl_group = dist.new_group(backend="gloo", timeout=tmo)

    grid = args.grid
    P = args.poses_per_gpu
    K = scene.intrinsics(WIDTH, HEIGHT)
    t_in = time.perf_counter()
    poses, depth = make_inputs(rank, world, P)
    log(f"[rank {rank}] inputs ready in {time.perf_counter() - t_in:.1f}s "
        f"(valid depth {float((depth > 0).mean()):.3f})")

    dev = torch.device("cuda", local_rank)
    stream = torch.cuda.current_stream(dev)
    vol = dmf_amd.VoxelVolume(local_rank)
    vol.set_stream(stream.cuda_stream)
    vol.setDimensions(-0.5, 0.5, -0.5, 0.5, -0.5, 0.5)
    vol.setVolumeSize(grid, grid, grid)
    vol.constructVolume()
    L = vol._L
    cam = _lib.make_camera(K, HEIGHT, WIDTH)
    prm = _lib.default_fuse_params(dmin_mm=scene.DEPTH_MIN_MM, dmax_mm=scene.DEPTH_MAX_MM)
    ncell = grid ** 3

    d_depth = torch.from_numpy(depth.view(np.int16)).to(dev)
    d_poses = torch.from_numpy(np.ascontiguousarray(poses, np.float32)).to(dev)
    # tiled counters padded to whole tile rows per rank: [hits | misses]
    npad = C.c_int64()
    _lib.check(L.dmf_fuse_counter_cells_padded(vol._h, world, C.addressof(npad)))
    npad = npad.value
    nlo = C.c_int64()
    _lib.check(L.dmf_fuse_logodds_cells_padded(vol._h, world, C.addressof(nlo)))
    logodds = torch.empty(nlo.value, dtype=torch.int16, device=dev)
    stats = torch.zeros(20, dtype=torch.int64, device=dev)  # 8 used; diagnostic builds add 7..19
    pcam, pprm = C.addressof(cam), C.addressof(prm)
    # Pipelined fusion (DMF_BENCH_PIPE=0 = serial): the frames are resident and
    # never rewritten, so their input stream is an idle one; each call's pass A then runs on
    # libdmf's staging stream beside the previous call's phase F.
    pipe = os.environ.get("DMF_BENCH_PIPE", "1") != "0"
    inp = torch.cuda.Stream(dev)
    torch.cuda.synchronize(dev)
    if pipe:
        _lib.check(L.dmf_fuse_set_input_stream(vol._h, inp.cuda_stream))
    # all fusion scratch allocated up front: the timed calls neither allocate nor sync
    _lib.check(L.dmf_fuse_reserve(vol._h, pcam, P, 0))

    # The step schedule (dmf_amd.schedule.run_steps, tested on CPU under random stream
    # orders): fuse on the compute stream; the merge of step i, then the zeroing of its
    # buffer for step i+2, on the comm stream, overlapping the fusion of step i+1 (two
    # counter buffers).  Merge = libdmf's
    # reduce-scatter / slab finalize / all-gather over torch's RCCL communicator (N > 1),
    # or the plain finalize (N = 1: no collective).
    merge_mode = os.environ.get("DMF_BENCH_MERGE", "rs")
    comm_ptr = None
    rccl = {"ranks": None, "merge": "finalize only (N = 1, no collective)" if world == 1 else None,
            "fallback_reason": None}
    if world > 1:
        dist.barrier()  # connects the RCCL communicator
        if backend != "nccl":
            rccl["fallback_reason"] = f"DMF_BENCH_BACKEND={backend}"
        elif merge_mode != "rs":
            rccl["fallback_reason"] = f"DMF_BENCH_MERGE={merge_mode}"
        elif not one_rccl_mapped():
            rccl["fallback_reason"] = "more than one librccl mapped: libdmf cannot use torch's communicator"
        if rccl["fallback_reason"] is None:
            try:
                comm_ptr = D.torch_comm_ptr(device=dev)
                nr, rk = C.c_int32(), C.c_int32()
                _lib.check(L.dmf_comm_shape(comm_ptr, C.addressof(nr), C.addressof(rk)))
                rccl["ranks"] = nr.value
                if nr.value != world or rk.value != rank:
                    raise RuntimeError(f"RCCL communicator spans {nr.value} ranks (rank {rk.value}), world {world} "
                                       f"rank {rank}")
            except (RuntimeError, AttributeError, TypeError, ValueError, _lib.DmfError) as ex:
                comm_ptr = None
                rccl["fallback_reason"] = f"torch's communicator not usable by libdmf: {ex}"
        # every rank takes the same merge path: a rank alone in libdmf's collectives would hang
        agree = torch.tensor([0 if comm_ptr is None else 1], dtype=torch.int32,
                             device=dev if backend == "nccl" else torch.device("cpu"))
        dist.all_reduce(agree, op=dist.ReduceOp.MIN)
        if int(agree.item()) == 0 and comm_ptr is not None:
            comm_ptr = None
            rccl["fallback_reason"] = "another rank cannot use torch's communicator from libdmf"
        if comm_ptr is not None:
            rccl["merge"] = ("libdmf dmf_fuse_merge_finalize_device: RCCL ncclReduceScatter(hits, misses) + slab "
                             "finalize + ncclAllGather(int16) on torch's communicator")
        else:
            merge_mode = "torch"
            rccl["merge"] = (f"fallback: torch.distributed all_reduce(sum) over {backend} + finalize of the "
                             "world-padded grid")
    bufs = [torch.zeros(2 * npad, dtype=torch.int32, device=dev) for _ in range(2)]
    rt = S.TorchRuntime(dev)  # the volume stays on the compute stream; merges name theirs
    ev = {}

    def clear(b):
        bufs[b].zero_()

    def fuse(b, i):
        c = bufs[b]
        _lib.check(L.dmf_fuse_depth_device(vol._h, pcam, d_depth.data_ptr(), d_poses.data_ptr(), P, pprm,
                                           c.data_ptr(), c.data_ptr() + 4 * npad, stats.data_ptr()))

    def merge(b, i):
        c = bufs[b]
        if comm_ptr is not None or world == 1:
            # N = 1: no communicator, the finalize alone (on the comm stream, behind fuse(i+1))
            try:
                D.merge_finalize_device(vol, c, pprm, logodds, comm_ptr, rt.lanes["comm"].cuda_stream)
            except _lib.DmfError as ex:  # only the merge's own failures may take the fallback
                raise MergeError(str(ex)) from ex
        else:
            # fallback: torch's all-reduce (RCCL, or gloo), issued on the comm lane (the current
            # stream here); the finalize of every slab of the world-padded counters follows it on
            # the same lane, so it reads the reduced counters and precedes the buffer's clear,
            # which run_steps also enqueues on the comm lane
            dist.all_reduce(c, op=dist.ReduceOp.SUM)
            _lib.check(L.dmf_fuse_finalize_slab_device(vol._h, c.data_ptr(), pprm, logodds.data_ptr(), world, -1,
                                                       rt.lanes["comm"].cuda_stream))

    def marks(i, name, lane):
        e = torch.cuda.Event(enable_timing=True)
        e.record(rt.lanes[lane])
        ev.setdefault(i, {})[name] = e

    # the merge (finalize) and clear of step i wait for step i+1's phase F to begin
    # (dmf_fuse_set_phase_event), so that they run beside the issue-bound phase F and not
    # beside the next call's passes A / B (DMF_BENCH_PHASE=0: right after step i's fusion).
    # At N > 1 the merge is RCCL's reduce-scatter / all-gather, whose kernels may not fit
    # beside phase F's persistent workgroups; it keeps the round-3 order unless
    # DMF_BENCH_PHASE=1 asks for the deferral there too.
    phase = None
    if os.environ.get("DMF_BENCH_PHASE", "1" if world == 1 else "0") != "0":
        fev = torch.cuda.Event()
        fev.record(stream)  # creates the event
        _lib.check(L.dmf_fuse_set_phase_event(vol._h, C.c_void_p(fev.cuda_event)))
        phase = lambda i: fev  # noqa: E731  (re-recorded by each fusion call)
    failed = None
    try:
        S.run_steps(rt, args.warmup, 2, clear, fuse, merge, phase=phase)
        torch.cuda.synchronize(dev)
    except MergeError as ex:  # a fusion error (NOMEM, RANGE ...) is not a merge failure: it raises
        if comm_ptr is None:
            raise
        failed = ex
    if comm_ptr is not None and world > 1:
        # the ranks agree on the fallback over the CPU group: one rank's failure moves every
        # rank to torch's all-reduce (a rank alone in libdmf's collective would wait for ever)
        flag = torch.tensor([0 if failed is None else 1], dtype=torch.int32)
        dist.all_reduce(flag, op=dist.ReduceOp.MAX, group=ctl_group)
        if int(flag.item()) and failed is None:
            failed = RuntimeError("another rank's libdmf RCCL merge failed in warmup")
    if failed is not None:
        # libdmf's RCCL merge failed: fall back to torch's all-reduce + finalize before anything
        # is timed, and say so in the line
        ex = failed
        log(f"[rank {rank}] libdmf RCCL merge failed in warmup ({ex}); falling back to torch all_reduce")
        comm_ptr, merge_mode = None, "torch"
        rccl["fallback_reason"] = f"libdmf RCCL merge failed in warmup: {ex}"
        rccl["merge"] = "fallback: torch.distributed all_reduce(sum) over RCCL + finalize of the world-padded grid"
        torch.cuda.synchronize(dev)
        S.run_steps(rt, max(args.warmup, 1), 2, clear, fuse, merge, phase=phase)
        torch.cuda.synchronize(dev)
    stats.zero_()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    S.run_steps(rt, args.steps, 2, clear, fuse, merge, marks=marks, phase=phase)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if phase is not None:  # the event is the bench's: unregister it before it goes away
        _lib.check(L.dmf_fuse_set_phase_event(vol._h, None))
    st = stats.cpu().numpy()
    ev = list(ev.values())
    nct = npad

    def seg(a, b):
        v = [r[a].elapsed_time(r[b]) for r in ev if a in r and b in r]
        return float(np.mean(v)) if v else 0.0
    clear_ms, fuse_ms, merge_ms = seg("z0", "z1"), seg("c1", "c2"), seg("a0", "a1")
    breakdown = {"clear": clear_ms, "fuse": fuse_ms, "merge": merge_ms,
                 "merge_kind": {"rs": "RCCL reduce-scatter(hits, misses) + slab finalize + all-gather(int16) "
                                      "(dmf_fuse_merge_finalize_device)",
                                "torch": f"torch {'RCCL' if backend == 'nccl' else backend} all-reduce(sum) + finalize"}[merge_mode] if world > 1
                 else "finalize (no collective at N=1)",
                 "schedule": "merge of step i, then the zeroing of its buffer for step i+2, on the comm stream overlap fuse of step i+1 (2 counter buffers)"
                             + ("; they wait for step i+1's phase F to begin (dmf_fuse_set_phase_event)" if phase else "")
                             + ("; pass A of fuse i+1 on libdmf's staging stream beside phase F of fuse i (the 'fuse' span is the "
                                "compute stream's: batch cut, B and F after waiting for that pass A)" if pipe else "")}
    # the merged grid of the timed steps (before the isolated re-timings below overwrite it)
    digest = hashlib.sha256(logodds[:ncell].cpu().numpy().tobytes()).hexdigest()[:16]
    # grid-wide streaming passes, priced separately: clear writes the
    # 2 tiled int32 counter arrays; finalize reads them and writes int16 log-odds.  In the timed
    # steps they run on the comm stream BESIDE the next call's phase F (by design), so their
    # event spans there are spans, not kernel durations: the *_isolated entries below re-time
    # each alone on the idle GPU after the timed region
    clear_bytes = 2 * 4 * nct
    fin_bytes = 10 * ncell

    def rate(ms_, nbytes, **kw):
        return dict({"ms": ms_, "bytes": nbytes, "GBps": nbytes / (ms_ * 1e-3) / 1e9 if ms_ else None,
                     "frac": nbytes / (ms_ * 1e-3) / 1e9 / HBM_PEAK_GBS if ms_ else None}, **kw)
    streaming = {"clear_span_overlapped": rate(clear_ms, clear_bytes, note="event span on the comm stream beside "
                                                                      "the next call's phase F (not a duration)")}
    if world == 1:
        streaming["finalize_span_overlapped"] = rate(merge_ms, fin_bytes, note="event span on the comm stream "
                                                                             "beside the next call's phase F")
    # isolated re-timing: each pass alone on the compute stream, GPU idle
    torch.cuda.synchronize(dev)
    niso = 20
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for _ in range(3):
        bufs[0].zero_()
    e0.record(stream)
    for _ in range(niso):
        bufs[0].zero_()
    e1.record(stream)
    torch.cuda.synchronize(dev)
    streaming["clear_isolated"] = rate(e0.elapsed_time(e1) / niso, clear_bytes,
                                       kernel="torch zero_ of the [hits | misses] int32 counters, alone")

    def fin_whole():
        _lib.check(L.dmf_fuse_finalize_slab_device(vol._h, bufs[1].data_ptr(), pprm, logodds.data_ptr(), world, -1,
                                                   stream.cuda_stream))
    for _ in range(3):
        fin_whole()
    e0.record(stream)
    for _ in range(niso):
        fin_whole()
    e1.record(stream)
    torch.cuda.synchronize(dev)
    streaming["finalize_isolated"] = rate(e0.elapsed_time(e1) / niso, fin_bytes,
                                          kernel="dmf::k_finalize over the whole grid (2 x int32 read + int16 "
                                                 "write per cell), alone")
    if st[3] != 0:  # pass B's device-side layout check (dmf_fuse_status): the counters are invalid
        raise RuntimeError(f"fusion layout check failed {st[3]} times")
    _lib.fuse_status(vol)  # raises DmfError(DMF_ERR_DEVICE_CHECK) if any call disagreed
    # how the device cut the calls (the per-volume budget may split a call)
    plan = _lib.fuse_plan(vol, cam, P)
    plan["batches_used_last_call"] = _lib.fuse_batches_used(vol) if plan.get("brick") else 1
    elapsed = D.max_over_ranks(elapsed, device=dev)
    updates, rays, hits = D.sum_over_ranks(st[:3], device=dev)

    # per-launch algorithmic bytes of the fusion launch (all its kernels), this rank
    upd_launch = float(st[0]) / args.steps
    bytes_launch = BYTES_PER_UPDATE * upd_launch + BYTES_PER_DEPTH * P * HEIGHT * WIDTH
    ms = elapsed / args.steps * 1e3
    serial_ms = None
    if pipe and args.serial_ref == "on":
        # pipelined calls overlap (pass A of call i+1 beside B and F of call i), so a call's own
        # event span is no duration: the fusion is priced over the whole step interval (which
        # also holds the overlapped finalize).  The serial call, timed alone, is reported beside.
        _lib.check(L.dmf_fuse_set_input_stream(vol._h, None))
        c = bufs[0]
        for _ in range(3):
            fuse(0, 0)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        nser = 50
        e0.record(stream)
        for _ in range(nser):
            fuse(0, 0)
        e1.record(stream)
        torch.cuda.synchronize(dev)
        serial_ms = e0.elapsed_time(e1) / nser
    # the time the fusion's algorithmic bytes are priced over: the step interval when the calls
    # are pipelined (they overlap: no per-call duration), the call's HIP-event span when serial
    step_ms = ms if pipe else fuse_ms
    achieved = bytes_launch / (step_ms * 1e-3) / 1e9
    golden = expected_digest(grid, P * world)

    result = None
    if rank == 0:
        secondary = {}
        if not args.no_secondary:
            secondary = secondary_reverse(vol, L, cam, dev, stream, d_depth, d_poses, P, K, poses, depth,
                                          cpu_poses=args.cpu_reverse_poses if world == 1 else 0,
                                          cpu_threads=args.cpu_threads, world=world)
        cpu = cpu_mt = cpu_ref = None
        if args.cpu_frames > 0 and world == 1:
            ups, rps, dt = cpu_baseline(K, poses, depth, args.cpu_frames, grid)
            cpu = {"value": ups, "unit": "ray-voxel updates/s", "cores": 1, "kind": "port",
                   "sample": f"oracle 3D-DDA fuse (this engine's spec, DESIGN.md 4: the reference has no DDA) of "
                             f"{args.cpu_frames} of the {P} frames ({WIDTH}x{HEIGHT}, {grid}^3), "
                             f"{dt:.1f}s single-threaded; Mrays/s {rps / 1e6:.3f}"}
            nt, nt_why = host_threads(args.cpu_threads)
            nf = min(P, max(4 * args.cpu_frames, nt))
            ups_mt, rps_mt, dt_mt = cpu_baseline(K, poses, depth, nf, grid, threads=nt)
            cpu_mt = {"value": ups_mt, "unit": "ray-voxel updates/s", "cores": nt, "kind": "port",
                      "threads_basis": nt_why,
                      "sample": f"oracle fuse (OpenMP rows, atomic counters) of {nf} of the {P} frames, "
                                f"{dt_mt:.1f}s on {nt} threads; Mrays/s {rps_mt / 1e6:.3f}"}
            cpu_ref = reference_fusion_baseline(K, poses, depth, P, grid)
        kname = _lib.kernel_name(vol)
        if kname.startswith("dmf::k_bk_fuse"):
            # brick-owned pipeline: step_ms spans every launch of the call
            # (A, the device-side batch cut, and per pose batch S, B, F)
            pipeline = ["dmf::k_bk_rays", "dmf::k_bk_batches", "dmf::k_bk_batch_counts", "dmf::k_bk_scan",
                        "dmf::k_bk_pairs", kname]
            diagnostics = {"pairs": int(st[4]) // args.steps, "parts": int(st[5]) // args.steps,
                           "flushed_cells": int(st[6]) // args.steps,
                           "updates_per_pair": float(st[0]) / max(float(st[4]), 1.0),
                           "updates_per_flushed_cell": float(st[0]) / max(float(st[6]), 1.0)}
            if st[7] > 0:  # diagnostic build (DMF_EXP_STATS): F wave blocks, lanes active, refills
                diagnostics.update({"f_blocks": int(st[7]) // args.steps, "f_refills": int(st[9]) // args.steps,
                                    "f_lane_util": float(st[8]) / max(64.0 * float(st[7]), 1.0),
                                    "b_replay_iters": int(st[18]) // args.steps,
                                    "b_lane_util": float(st[19]) / max(64.0 * float(st[18]), 1.0),
                                    "f_wave_cycles": {"refill": int(st[10]) // args.steps, "walk": int(st[11]) // args.steps,
                                                      "flush": int(st[12]) // args.steps,
                                                      "part_barrier": int(st[15]) // args.steps,
                                                      "refill_decode": int(st[16]) // args.steps,
                                                      "refill_prefetch": int(st[17]) // args.steps,
                                                      "lifetime_sum": int(st[14]) // args.steps,
                                                      "lifetime_max_wave": int(st[13])}})
        else:
            pipeline = [kname]
            diagnostics = {"lds_rounds": int(st[4]), "fallback_rounds": int(st[5]),
                           "flushed_cell_atomics": int(st[6]),
                           "updates_per_flushed_atomic": float(st[0]) / max(float(st[6]), 1.0)}
        result = {
            "metric": f"ray-voxel updates/sec (3D-DDA log-odds fusion, {grid}^3 grid, {WIDTH}x{HEIGHT} depth)",
            "value": updates / elapsed,
            "unit": "ray-voxel updates/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "int32",  # exact integer DDA (int32 walk state) and int32 hit/miss counters
            "data": "synthetic: analytic sphere+box+ground scene rendered to uint16 mm depth, Fibonacci poses r=0.7m",
            "config": {"workload": f"{workload_name(grid, P, world)}: {P} poses/GPU x {WIDTH}x{HEIGHT} depth -> "
                                   f"{grid}^3 int16 "
                                   f"log-odds (int32 hit/miss counters)",
                       "grid": grid, "image": f"{WIDTH}x{HEIGHT}", "poses_per_gpu": P, "global_poses": P * world,
                       "parallelism": f"pose-sharded dp{world}" + (
                           " + RCCL reduce-scatter / all-gather merge (libdmf)" if merge_mode == "rs" and world > 1
                           else f" + {'RCCL' if backend == 'nccl' else backend} all-reduce(sum) merge" if world > 1
                           else "")},
            "mrays_per_s": rays / elapsed / 1e6,
            "fuse_diagnostics": diagnostics,
            "fuse_plan": plan,
            "updates_per_ray": updates / max(rays, 1.0),
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": None,
                         "basis": "effective (algorithmic): SURVEY.md 8d bytes, 4 B per cell update + 2 B per depth "
                                  "pixel, " + ("over the step interval of the pipelined fusion (elapsed / steps: pass A "
                                               "of call i+1 runs beside passes B and F of call i, DESIGN.md 5.10)"
                                               if pipe else "over the fusion launch's HIP-event time")
                                  + "; the brick pipeline accumulates in LDS, so these bytes are a price, not its "
                                    "HBM traffic",
                         "measured_frac": None, "traffic_source": None,
                         "kernel": kname, "step_ms": step_ms,
                         "step_ms_basis": ("elapsed / steps of the pipelined calls (each step also holds the "
                                           "overlapped finalize)" if pipe else "HIP events around the serial fusion call"),
                         "kernel_avg_ms": None,  # per-kernel averages from a rocprofv3 --kernel-trace child (attach_pmc)
                         "f_kernel_ms": None,
                         "companion": None,      # the valu-issue bound that binds the pipeline (attach_pmc)
                         "pipeline": pipeline,
                         "pipelined": pipe, "serial_call_ms": serial_ms,
                         "serial_call_frac": (bytes_launch / (serial_ms * 1e-3) / 1e9 / HBM_PEAK_GBS
                                              if serial_ms else None),
                         "updates_per_launch": upd_launch, "algorithmic_bytes_per_launch": bytes_launch},
            "cpu_baseline": cpu,
            "cpu_baseline_multicore": cpu_mt,
            # the reference's own fusion (integratePointCloud, one voxel per point) on the same frames
            "cpu_baseline_reference": cpu_ref,
            "host_cores": host_cores(),
            "step_breakdown_ms": breakdown,
            "streaming": streaming,
            "secondary": secondary,
            # the merged grid after the last step (the same poses every step) against the oracle's
            # digest of the same global poses (tests/golden/gen_fusion_digests.py): the line checks
            # its own exactness at N = 1 and, over the merge, at N > 1
            "logodds_digest": digest,
            "digest_expected": golden["logodds_digest"] if golden else None,
            "digest_match": (digest == golden["logodds_digest"]) if golden else None,
            "digest_source": (f"oracle (CPU restatement) fusion of the {P * world} global poses, "
                              f"tests/golden/fusion_digests.json[{golden['key']}]") if golden else
                             "no committed oracle digest for this workload",
            "rccl": rccl,
        }
    if dist.is_initialized():
        dist.barrier()
        dist.destroy_process_group()
    vol.close()
    del bufs, logodds, d_depth
    torch.cuda.empty_cache()
    if result is not None and world == 1 and args.pmc == "auto":
        attach_pmc(result, pmc_measure(args, args.pmc_dir))
    if result is not None:
        os.write(json_fd, (json.dumps(result) + "\n").encode())


def attach_pmc(result, pmc):
    """Fill the bench line's measured fields from a pmc_measure() run: HBM traffic per
    fusion launch (all kernels of the fusion call), VALU/SALU instructions per launch, and
    the issue-bound pricing of the secondary march kernels."""
    rf = result["roofline"]
    if not pmc:
        rf["traffic_source"] = "not measured (rocprofv3 unavailable or a PMC pass failed)"
        return
    kt = pmc.pop("__kernel_trace__", {}) or {}
    fk = [k for k in pmc if k.startswith(("dmf::k_bk_", "dmf::k_fuse"))]
    calls = 1  # the child run makes one fusion call (steps 1, warmup 0)
    fetch, write = pmc_total(pmc, fk, "FETCH_SIZE"), pmc_total(pmc, fk, "WRITE_SIZE")
    traffic = 1024.0 * (2.0 * fetch + write) / calls
    valu = pmc_total(pmc, fk, "SQ_INSTS_VALU") / calls
    rf["traffic"] = traffic
    rf["measured_frac"] = traffic / (rf["step_ms"] * 1e-3) / 1e9 / HBM_PEAK_GBS
    if kt:
        rf["kernel_avg_ms"] = {k: round(v["avg_ms"], 4) for k, v in sorted(kt.items())}
        fkey = [k for k in kt if k.startswith("dmf::k_bk_fuse") or k.startswith("dmf::k_fuse_l")]
        if fkey:
            rf["f_kernel_ms"] = kt[fkey[0]]["avg_ms"]
            rf["f_kernel"] = fkey[0]
        rf["kernel_avg_source"] = ("rocprofv3 --kernel-trace --stats of the same workload, 20 steps in the timed "
                                   "mode (child run): passes A and B run beside the previous call's F when "
                                   "pipelined, so their averages include the stretch")
    fvalu = pmc_per_dispatch(pmc, rf.get("f_kernel") or "", "SQ_INSTS_VALU") if rf.get("f_kernel") else None
    flds = pmc_per_dispatch(pmc, rf.get("f_kernel") or "", "SQ_INSTS_LDS") if rf.get("f_kernel") else None
    fconf = pmc_per_dispatch(pmc, rf.get("f_kernel") or "", "SQ_LDS_BANK_CONFLICT") if rf.get("f_kernel") else None
    rf["companion"] = {
        "bound": "valu-issue", "achieved": valu / (rf["step_ms"] * 1e-3), "peak": VALU_PEAK_WIPS,
        "unit": "wave-instr/s", "frac": valu / (rf["step_ms"] * 1e-3) / VALU_PEAK_WIPS,
        "valu_per_call": valu, "lane_slots_per_update": valu * 64.0 / max(rf["updates_per_launch"], 1.0),
        "f_valu_per_launch": fvalu,
        "f_frac": (fvalu / (rf["f_kernel_ms"] * 1e-3) / VALU_PEAK_WIPS) if fvalu and rf.get("f_kernel_ms") else None,
        # phase F is bound by its LDS adds as much as by its VALU (at the margin one
        # LDS add costs about 5.8 VALU): its LDS instructions against one ds_add per 4 cycles per CU
        "f_lds_per_launch": flds, "f_lds_bank_conflict_cycles": fconf,
        "f_lds_frac": (flds / (rf["f_kernel_ms"] * 1e-3) / LDS_ADD_PEAK_WIPS) if flds and rf.get("f_kernel_ms") else None,
        "basis": "what binds the pipeline: SQ_INSTS_VALU of every fusion kernel per call (PMC child) over the step "
                 "interval, vs 1024 SIMD-32 x one wave64 VALU instruction per 2 cycles at 2.4 GHz"}
    rf["traffic_source"] = ("rocprofv3 --pmc FETCH_SIZE | WRITE_SIZE passes of this configuration (child runs after "
                            "the timed region), (2 x FETCH_SIZE + WRITE_SIZE) x 1024 per fusion call, summed over "
                            + ", ".join(sorted(fk)))
    rf["per_kernel_hbm_bytes"] = {k: 1024.0 * (2.0 * pmc_total(pmc, [k], "FETCH_SIZE") + pmc_total(pmc, [k], "WRITE_SIZE"))
                                  / calls for k in sorted(fk)}
    rf["valu_per_launch"] = valu
    rf["valu_issue_frac"] = rf["companion"]["frac"]
    rf["valu_lane_slots_per_update"] = valu * 64.0 / max(rf["updates_per_launch"], 1.0)
    sec = result.get("secondary") or {}
    for name, prefixes in (("reverse_ray_trace_fast", ("dmf::k_reverse_x", "dmf::k_reverse_q")),
                           ("forward_first_hits", ("dmf::k_forward",))):
        if name not in sec:
            continue
        ks = [k for p_ in prefixes for k in pmc if k == p_ or k.startswith(p_ + "<")]
        if ks:
            sec[name]["roofline"] = issue_roofline(pmc, ks[0], sec[name].get("kernel_ms") or sec[name]["ms_per_batch"])


def reverse_cpu_baseline(grid, K, poses, pts, nrm, n_threads, n_poses):
    """The reference's own hot function on the host: oracle reverseRayTraceFast, a line-by-line
    restatement in the reference's layout (vector<vector<vector<Voxel*>>>, unordered_set
    lookups, 1 mm march) WITH the dead getNeighborHashes(K=5) work the reference does per
    voxel (RayTracingEngine.hpp:136-226, 170-171), over the same integrated volume: one pose
    single-threaded, then n_poses poses over n_threads threads (one pose per thread; the
    reference itself is single-threaded).  Unit: voxel-pose evaluations/s (occupied voxels x
    poses / s), the same as the GPU line beside it."""
    from concurrent.futures import ThreadPoolExecutor
    from oracle import oracle as O
    ov = O.Volume()
    ov.setDimensions(-0.5, 0.5, -0.5, 0.5, -0.5, 0.5)
    ov.setVolumeSize(grid, grid, grid)
    ov.constructVolume()
    ov.integratePointCloud(pts, nrm)
    V = len(ov.occupied_cells_)
    eng = O.Engine(K)
    t0 = time.perf_counter()
    _, good0 = eng.reverseRayTraceFast(ov, poses[0], False, dead_work=True)
    dt1 = time.perf_counter() - t0
    out = {"value": V / dt1, "unit": "voxel-pose evaluations/s", "cores": 1, "kind": "port",
           "_pose0_good": good0, "_occupied": ov.occupied_cells_,
           "sample": f"oracle reverseRayTraceFast (reference layout, dead getNeighborHashes kept) of 1 of the "
                     f"{len(poses)} poses over the same {V}-voxel volume, {dt1:.1f}s single-threaded"}
    if n_poses > 0 and n_threads > 1:
        sel = [poses[i % len(poses)] for i in range(n_poses)]
        t0 = time.perf_counter()
        with ThreadPoolExecutor(n_threads) as ex:  # ctypes calls release the GIL
            list(ex.map(lambda T: eng.reverseRayTraceFast(ov, T, False, dead_work=True), sel))
        dtm = time.perf_counter() - t0
        out["multicore"] = {"value": V * n_poses / dtm, "unit": "voxel-pose evaluations/s", "cores": n_threads,
                            "kind": "port", "sample": f"{n_poses} poses on {n_threads} threads (one pose per "
                                                      f"thread), {dtm:.1f}s"}
    return out


MARCH_GOLDEN = os.path.join(ROOT, "tests", "golden", "march_digests.json")


def march_digest(a):
    """sha256 of an array's bytes, first 16 hex digits (tests/golden/gen_march_digests.py)."""
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()[:16]


def expected_march(grid, P, n_int, Vc, world):
    """The oracle's digests of this run's secondary workload (tests/golden/gen_march_digests.py),
    or None: only the N = 1 pose set (rank 0's poses at N > 1 are another shard) was generated."""
    if world != 1:
        return None
    try:
        table = json.load(open(MARCH_GOLDEN))
    except (OSError, ValueError):
        return None
    for key, e in table.items():
        if (e["grid"], e["image"], e["poses"], e["seed"], e["integrated_frames"], e["costmap_centres"]) == (
                grid, f"{WIDTH}x{HEIGHT}", P, 1234, n_int, Vc):
            return dict(e, key=key)
    return None


def secondary_reverse(vol, L, cam, dev, stream, d_depth, d_poses, P, K, poses_h, depth_h, n_int=16, cpu_poses=16,
                      cpu_threads=0, world=1):
    """reverseRayTraceFast (RayTracingEngine.hpp:136-226) throughput for the same poses over a
    volume integrated from n_int back-projected frames (march samples/s, voxel-rays/s), with
    the reference-layout CPU port timed beside it (cpu_poses > 0), the forward march's first
    hits and the run_tsp cost map; each output is checked against the oracle's digest of the
    same workload (tests/golden/march_digests.json) and the reverse CPU leg's pose-0 list
    against the GPU's."""
    import ctypes as C
    H, W = HEIGHT, WIDTH
    n_int = min(n_int, P)  # (a rank with fewer frames integrates all of them)
    xyz = torch.empty((n_int, H, W, 3), dtype=torch.float32, device=dev)
    _lib.check(L.dmf_backproject_device(vol._h, C.addressof(cam), d_depth.data_ptr(), d_poses.data_ptr(), n_int,
                                        xyz.data_ptr()))
    valid = (d_depth[:n_int].view(torch.int16) > 0).reshape(-1)
    pts = xyz.reshape(-1, 3)[valid].contiguous()
    hp = d_poses[:n_int].cpu().numpy()
    nrm = np.concatenate([scene.render(K, W, H, hp[i])[1].reshape(-1, 3) for i in range(n_int)])
    d_nrm = torch.from_numpy(nrm).to(dev).reshape(-1, 3)[valid].contiguous()
    vol.integrate_device(pts.data_ptr(), d_nrm.data_ptr(), pts.shape[0])
    V = vol.info()["num_occupied"]
    words = (V + 63) // 64
    good = torch.empty(P * words, dtype=torch.int64, device=dev)
    st = torch.zeros(16, dtype=torch.int64, device=dev)  # [samples, rays] (+ diagnostic-build counters)

    def run():
        _lib.check(L.dmf_reverse_visibility_device(vol._h, C.addressof(cam), d_poses.data_ptr(), P, 0, None,
                                                   good.data_ptr(), st.data_ptr()))
    f0 = torch.cuda.Event(enable_timing=True)
    f1 = torch.cuda.Event(enable_timing=True)
    f0.record(stream)
    run()  # first call after integration also builds the brick distance field
    f1.record(stream)
    torch.cuda.synchronize(dev)
    first_ms = f0.elapsed_time(f1)
    st.zero_()
    e0 = torch.cuda.Event(enable_timing=True)
    e1 = torch.cuda.Event(enable_timing=True)
    reps = 2
    e0.record(stream)
    for _ in range(reps):
        run()
    e1.record(stream)
    torch.cuda.synchronize(dev)
    ms = e0.elapsed_time(e1) / reps
    s = st.cpu().numpy() / reps
    bytes_launch = 2.0 * s[0]  # 2 B (int16-equivalent read) per query-only march sample
    # forward depth-plane march (RayTracingEngine.hpp:280-308 semantics), dense 640x480,
    # all P poses in one launch: first occupied sample per pixel
    kbuf = torch.empty(P * H * W, dtype=torch.int32, device=dev)
    sbuf = torch.empty(P * H * W, dtype=torch.int32, device=dev)
    fst = torch.zeros(1, dtype=torch.int64, device=dev)

    def fwd():
        _lib.check(L.dmf_forward_first_hits_device(vol._h, C.addressof(cam), d_poses.data_ptr(), P, 10, 10, 1, 1,
                                                   kbuf.data_ptr(), sbuf.data_ptr(), fst.data_ptr()))
    fwd()
    torch.cuda.synchronize(dev)
    fst.zero_()
    g0 = torch.cuda.Event(enable_timing=True)
    g1 = torch.cuda.Event(enable_timing=True)
    g0.record(stream)
    fwd()
    g1.record(stream)
    torch.cuda.synchronize(dev)
    fwd_ms = g0.elapsed_time(g1)
    fwd_samples = float(fst.cpu().numpy()[0])
    forward = {"rays": P * H * W, "ms_per_batch": fwd_ms, "march_samples_per_s": fwd_samples / (fwd_ms * 1e-3),
               "mrays_per_s": P * H * W / (fwd_ms * 1e-3) / 1e6,
               "roofline": None,  # issue-bound pricing from the PMC passes (attach_pmc)
               "algorithmic_bytes_per_launch": 2.0 * fwd_samples}
    # set-cover consumer (Algorithms.hpp:38-86) over the same good sets
    sel = np.zeros(P, np.int32)
    nsel = C.c_int32()
    t0 = time.perf_counter()
    _lib.check(L.dmf_greedy_set_cover_masks_device(vol._h, good.data_ptr(), P, words, 5, sel.ctypes.data,
                                                   C.addressof(nsel)))
    cover_ms = (time.perf_counter() - t0) * 1e3
    # Planner::run_tsp cost map (tests/CameraPathGen.cpp:310-331): willCollide over all
    # ordered pairs of 1024 camera centres on a 0.45 m sphere inside the volume (the
    # createCameraLocationsFromSphere layout), one launch
    Vc = 1024
    cp = scene.sphere_centres(Vc)
    d_cp = torch.from_numpy(cp).to(dev)
    cmap = torch.empty((Vc, Vc), dtype=torch.int32, device=dev)

    def costmap():
        _lib.check(L.dmf_collision_cost_map_device(vol._h, d_cp.data_ptr(), Vc, cmap.data_ptr()))
    costmap()
    torch.cuda.synchronize(dev)
    h0 = torch.cuda.Event(enable_timing=True)
    h1 = torch.cuda.Event(enable_timing=True)
    h0.record(stream)
    costmap()
    h1.record(stream)
    torch.cuda.synchronize(dev)
    cm_ms = h0.elapsed_time(h1)
    collided = int((cmap == 0x7FFFFFFF).sum().item())
    # exactness at the timed size: digests of the GPU outputs against the oracle's
    # (tests/golden/gen_march_digests.py) -- the occupied list, the good masks (P x words
    # uint64 over occupied_cells_ slots), the forward (k, slot) maps, the cost map
    occ = vol.occupied_cells_
    got = {"occupied_digest": march_digest(np.asarray(occ, np.uint64)),
           "reverse_good_digest": march_digest(good.cpu().numpy().view(np.uint64).reshape(P, words)),
           "forward_k_digest": march_digest(kbuf.cpu().numpy()),
           "forward_slot_digest": march_digest(sbuf.cpu().numpy()),
           "costmap_digest": march_digest(cmap.cpu().numpy())}
    gold = expected_march(vol.dims[0], P, n_int, Vc, world)

    def check(*keys):
        d = {k: got[k] for k in keys}
        d["digest_match"] = all(got[k] == gold[k] for k in keys) if gold else None
        d["digest_source"] = (f"oracle (CPU restatement) on the same workload, tests/golden/march_digests.json"
                              f"[{gold['key']}]") if gold else "no committed oracle digest for this workload"
        return d
    rev_cpu = None
    if cpu_poses > 0:
        rev_cpu = reverse_cpu_baseline(vol.dims[0], K, poses_h, pts.cpu().numpy(), d_nrm.cpu().numpy(),
                                       host_threads(cpu_threads)[0], cpu_poses)
        # per-run check, for free: the CPU leg's pose-0 good list (the oracle on the volume it
        # integrated from the same points) against the GPU's pose-0 mask, and the two
        # occupied_cells_ lists
        g0 = good[:words].cpu().numpy().view(np.uint64)
        slots = np.nonzero(np.unpackbits(g0.view(np.uint8), bitorder="little")[:V])[0]
        gpu_list = np.asarray(occ, np.uint64)[slots]
        ref_occ = rev_cpu.pop("_occupied")
        ref_list = np.asarray(rev_cpu.pop("_pose0_good"), np.uint64)
        rev_cpu["pose0_list_match"] = bool(np.array_equal(gpu_list, ref_list) and
                                           np.array_equal(np.asarray(occ, np.uint64), np.asarray(ref_occ, np.uint64)))
        rev_cpu["pose0_good"] = int(ref_list.size)
    forward.update(check("forward_k_digest", "forward_slot_digest"))
    return {"greedy_set_cover": {"candidates": P, "selected": int(nsel.value), "ms": cover_ms},
            "collision_cost_map": {"centres": Vc, "pairs": Vc * Vc, "collided_pairs": collided, "ms": cm_ms,
                                   "pairs_per_s": Vc * Vc / (cm_ms * 1e-3), **check("costmap_digest")},
            "forward_first_hits": forward,
            "reverse_ray_trace_fast": {
        "occupied_voxels": int(V), "poses": P, "ms_per_batch": ms,
        "first_call_ms": first_ms, "note": "first call after integration includes the brick distance field build",
        "march_samples_per_s": float(s[0]) / (ms * 1e-3), "voxel_rays_per_s": float(s[1]) / (ms * 1e-3),
        "voxel_pose_evaluations_per_s": float(V) * P / (ms * 1e-3),
        "cpu_baseline": rev_cpu,
        "roofline": None,  # issue-bound pricing from the PMC passes (attach_pmc); the march reads an
                           # L2-resident bitmask, so SURVEY 8d's 2 B per sample is reported, not a bound:
        "algorithmic_bytes_per_launch": bytes_launch,
        **check("occupied_digest", "reverse_good_digest"),
        **({"diagnostics": dict(zip(REV_DIAG, (float(x) for x in s[2:2 + len(REV_DIAG)])))} if s[2:].any() else {})}}


# counters 2.. of the DMF_EXP_STATS library's reverse march (per batch; dmf_trace.hip DMF_RS)
REV_DIAG = ["centroid_cell_samples", "stepped_samples", "jump_tries", "jumps", "jumped_samples", "collided",
            "exited", "marched_rays", "burst_iterations", "burst_active_lanes", "jump_too_short"]


if __name__ == "__main__":
    main()
