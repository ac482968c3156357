"""The per-step fusion schedule of the pose-sharded engine, written once
against a small stream runtime so the same code drives the GPU (torch/HIP streams and
events) and a CPU simulator that executes the enqueued work in random stream-consistent
orders (gloo collectives inside).

One step on one rank:
  compute lane:  [wait until buffer b's previous merge + clear are done] fuse(b, i)
  comm lane:     [wait fuse(b, i)] merge(b, i) (reduce-scatter + slab finalize +
                 all-gather, or all-reduce + finalize) -> clear(b) for step i + nbuf
Counters are multi-buffered, so the merge of step i and the zeroing of its buffer overlap
the fusion of step i+1.  A buffer's first use in a run is cleared on the compute lane, so
K steps do exactly K clears, K fusions and K merges; the last merge is waited for before
the schedule returns (it is inside the timed region).
"""
from __future__ import annotations

import random


class TorchRuntime:
    """HIP streams via torch: enqueue() calls the function on the host with the lane's
    stream current, so the native calls it makes go to that stream (they take their
    stream from the volume: the caller's `bind(lane)` hook sets it)."""

    def __init__(self, device, bind=None):
        import torch
        self.torch = torch
        self.device = device
        self.bind = bind
        self.lanes = {"compute": torch.cuda.current_stream(device), "comm": torch.cuda.Stream(device)}

    def enqueue(self, lane, fn):
        s = self.lanes[lane]
        with self.torch.cuda.stream(s):
            if self.bind is not None:
                self.bind(s)
            fn()

    def record(self, lane):
        e = self.torch.cuda.Event()
        e.record(self.lanes[lane])
        return e

    def wait(self, lane, event):
        self.lanes[lane].wait_event(event)

    def drain(self):
        if self.bind is not None:
            self.bind(self.lanes["compute"])


class _SimEvent:
    __slots__ = ("done",)

    def __init__(self):
        self.done = False


class SimRuntime:
    """CPU stand-in for streams: each lane is a FIFO of work; drain() runs, at random,
    any lane whose head is ready (an event wait is ready once the event's record ran).
    A schedule that forgets a wait computes wrong results under some orders."""

    def __init__(self, seed=0):
        self.rng = random.Random(seed)
        self.q = {"compute": [], "comm": []}

    def enqueue(self, lane, fn):
        self.q[lane].append(("run", fn))

    def record(self, lane):
        e = _SimEvent()
        self.q[lane].append(("record", e))
        return e

    def wait(self, lane, event):
        self.q[lane].append(("wait", event))

    def drain(self):
        while any(self.q.values()):
            ready = [k for k, v in self.q.items() if v and (v[0][0] != "wait" or v[0][1].done)]
            if not ready:
                raise RuntimeError("schedule deadlock: every lane waits on an unrecorded event")
            lane = self.rng.choice(ready)
            kind, arg = self.q[lane].pop(0)
            if kind == "run":
                arg()
            elif kind == "record":
                arg.done = True


def run_steps(rt, nsteps, nbuf, clear, fuse, merge, marks=None, reuse_wait=True, phase=None):
    """Enqueue `nsteps` steps on runtime `rt` and wait for the last merge.

    clear(b), fuse(b, i), merge(b, i) enqueue (or, on the simulator, perform) the work of
    step i on counter buffer b = i % nbuf.  marks(i, name, lane), if given, is called at
    the step's phase boundaries (z0, z1 around the clear that prepares step i's buffer, on
    whichever lane runs it; c1, c2 around the fusion on compute; a0, a1 around the merge
    on comm) for timing.  reuse_wait=False drops the buffer-reuse dependency (tests show it
    is needed).

    phase(i), if given, returns an event that fuse(b, i) recorded when its phase F begins
    (dmf_fuse_set_phase_event): the merge of step i - 1 (and the clear behind it) then also
    waits for it, so that this HBM-bound work runs beside step i's issue-bound phase F rather
    than beside its passes A / B; the last step's merge follows its fusion."""
    def mark(i, name, lane):
        if marks:
            marks(i, name, lane)

    merged = [None] * nbuf
    last = None

    def enqueue_merge(b, i, fused, after=None):
        nonlocal last
        rt.wait("comm", fused)
        if after is not None:
            rt.wait("comm", after)
        mark(i, "a0", "comm")
        rt.enqueue("comm", lambda b=b, i=i: merge(b, i))
        mark(i, "a1", "comm")
        if i + nbuf < nsteps:  # zero the buffer for step i + nbuf behind its merge
            mark(i + nbuf, "z0", "comm")
            rt.enqueue("comm", lambda b=b: clear(b))
            mark(i + nbuf, "z1", "comm")
        merged[b] = last = rt.record("comm")

    if phase is not None and nbuf < 2:
        # the deferred merge of step i is enqueued after fuse(i + 1), which would add into
        # the same single buffer before the merge read it
        raise ValueError("run_steps: a phase-deferred merge needs at least 2 counter buffers")
    pending = None  # (b, i, fused) of the step whose merge waits for the next phase F
    for i in range(nsteps):
        b = i % nbuf
        if reuse_wait and merged[b] is not None:
            rt.wait("compute", merged[b])
        if i < nbuf:  # the buffer's first use in this run
            mark(i, "z0", "compute")
            rt.enqueue("compute", lambda b=b: clear(b))
            mark(i, "z1", "compute")
        mark(i, "c1", "compute")
        rt.enqueue("compute", lambda b=b, i=i: fuse(b, i))
        mark(i, "c2", "compute")
        fused = rt.record("compute")
        if phase is None:
            enqueue_merge(b, i, fused)
        else:
            ph = phase(i)
            if pending is not None:
                enqueue_merge(*pending, after=ph)
            pending = (b, i, fused)
    if pending is not None:
        enqueue_merge(*pending)
    if last is not None:
        rt.wait("compute", last)
    rt.drain()
