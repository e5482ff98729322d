"""Distributed data parallel: bucketed gradient all-reduce overlapped with backward.

Replaces ``torch.nn.parallel.DistributedDataParallel`` as used by the reference
(``resnet50_test.py:716``: default 25 MB buckets, ``broadcast_buffers=True``; survey P5,
X2-X4) with a reducer designed around the flat gradient buffer (``utils/flat.py``):

* buckets are contiguous slices of the flat fp32 gradient (gradient-as-bucket-view:
  no flatten/unflatten copies), in reverse registration order = backward order;
* each parameter's post-accumulate-grad hook counts down its bucket; a full bucket is
  launched immediately as an async ``all_reduce`` on RCCL's stream (backend ``nccl`` is
  RCCL on ROCm), so communication overlaps the rest of backward;
* ``finish()`` (call after ``backward``) launches any bucket left (unused params) and
  makes the compute stream wait on RCCL — no host blocking on GPU;
* with the backward captured as HIP graphs (the ResNet engine's, or any autograd backward
  under ``parallel/graphs.SegmentedStep``), the capture is cut where a bucket completes and
  that bucket's all-reduce is launched between the replayed segments, so overlap survives
  graph replay;
* averaging uses ``ReduceOp.AVG`` on RCCL (no extra scaling pass), ``SUM`` + scale on
  gloo; optional bf16 wire format halves bytes on xGMI.

Bucket sizing for MI355X: an 8-GPU node connects every GPU to every other by one xGMI
link (7 x ~153 GB/s per GPU).  RCCL's multi-channel algorithms spread a large message
over all links, so per-bucket cost is latency-dominated below a few MB and bandwidth-
dominated above; the exposed cost is the LAST bucket.  Round 2 chose a 1 MB first bucket
(communication starts after the classifier/last stage) then 8 MB buckets -- ResNet-50's
89.6 MB fp32 gradient as ~12 buckets, an exposed tail of ~8 MB (~15 µs at 7-link bandwidth).
Measured against that (round 3, ``bench.py --ddp`` = this reducer over a world-1 RCCL group,
so every cost but the transfer itself): each bucket costs ~25 µs of graph cut + collective
launch on the GPU timeline at ResNet-50 batch 128 -- 12 buckets 5.95 ms/step, 6 buckets
5.78, 3 buckets 5.74, no reducer 5.52 (``profiles/r3s3/ddp_world1_*.json``).  The ResNet
trainer and the bench therefore default to 25 MB buckets (after the 1 MB first one): ~0.17 ms
less per step than 8 MB against ~0.1 ms more exposed tail at 8 GPUs.
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from ..ops import _native
from ..utils.flat import FlatParams
from . import graphs


def plan_buckets_py(sizes, first_cap, cap):
    """Python twin of the native ``plan_buckets`` (csrc/runtime/runtime.cpp)."""
    buckets, cur, acc, limit = [], [], 0, first_cap
    for i in range(len(sizes) - 1, -1, -1):
        cur.append(i)
        acc += sizes[i]
        if acc >= limit:
            buckets.append(cur)
            cur, acc, limit = [], 0, cap
    if cur:
        buckets.append(cur)
    return buckets


def plan_buckets(sizes, first_cap, cap):
    nat = _native.load()
    if nat is not None:
        return [list(b) for b in nat.plan_buckets(list(map(int, sizes)), int(first_cap), int(cap))]
    return plan_buckets_py(sizes, first_cap, cap)


class BucketReducer:
    def __init__(self, flat: FlatParams, module=None, process_group=None, bucket_mb: float = 25.0,
                 first_bucket_mb: float = 1.0, comm_dtype: torch.dtype | None = None,
                 broadcast_buffers: bool = True, broadcast_init: bool = True):
        self.flat = flat
        self.module = module
        self.pg = process_group
        self.ws = dist.get_world_size(process_group)
        self.comm_dtype = comm_dtype
        self.broadcast_buffers = broadcast_buffers
        backend = dist.get_backend(process_group)
        self.use_avg = backend == "nccl"
        # flat slots are in REVERSE registration order already; plan over registration
        # order so the planner's "reverse" walk yields flat (=backward) order.
        slots = flat.slots[::-1]
        sizes = [s.numel * 4 for s in slots]
        plan = plan_buckets(sizes, int(first_bucket_mb * 2**20), int(bucket_mb * 2**20))
        self.buckets = []  # (start, end, [slot indices in flat order])
        n_slots = len(slots)
        for b in plan:
            flat_idx = [n_slots - 1 - i for i in b]
            start = min(flat.slots[i].offset for i in flat_idx)
            last = max(flat_idx)
            end = flat.slots[last].offset + flat.slots[last].numel
            end = min((end + 63) // 64 * 64, flat.numel)
            self.buckets.append((start, end, flat_idx))
        # make buckets tile the buffer exactly (padding elements travel with a bucket)
        for k in range(len(self.buckets) - 1):
            s, _, idx = self.buckets[k]
            self.buckets[k] = (s, self.buckets[k + 1][0], idx)
        if self.buckets:
            s, _, idx = self.buckets[-1]
            self.buckets[-1] = (s, flat.numel, idx)
        self.bucket_of = {}
        for b, (_, _, idx) in enumerate(self.buckets):
            for i in idx:
                self.bucket_of[id(flat.slots[i].param)] = b
        self.pending = [len(idx) for (_, _, idx) in self.buckets]
        self.ready = set()  # parameters signalled ready this step
        self.works = [None] * len(self.buckets)
        # reduced-precision wire format: ONE persistent buffer shaped like the flat gradient,
        # each bucket a view of it (no per-step allocation; the cast in and out are the only
        # extra passes)
        self.wire = None
        if comm_dtype is not None and comm_dtype != flat.grad.dtype:
            self.wire = torch.empty(flat.numel, device=flat.grad.device, dtype=comm_dtype)
        self.cast = [False] * len(self.buckets)
        self.in_graph = set()  # buckets whose all-reduce was captured into a backward graph
        from ..ops.resnet_fused import register_grad_ready_hook
        # autograd-managed params fire the post-accumulate hook; params whose gradient the
        # fused ResNet engine writes directly fire the engine's grad-ready hook
        self._hooks = [s.param.register_post_accumulate_grad_hook(self._hook) for s in flat.slots]
        self._hooks += [register_grad_ready_hook(s.param, self._hook, deferrable=True) for s in flat.slots]
        self.enabled = True
        if broadcast_init:
            self.broadcast_parameters()

    # ------------------------------------------------------------------ hooks
    def _hook(self, p, defer=False):
        """Gradient of ``p`` is final.  ``defer`` (the engine is capturing its backward into
        HIP graphs): do the bookkeeping, return the launch as a callable instead.  Under any
        other graph recording (parallel/graphs.py, e.g. an autograd backward being captured)
        the capture is cut here and the launch runs between the replayed segments."""
        if not self.enabled:
            return None
        if id(p) in self.ready:
            # a second readiness signal for the same parameter in one step (autograd's
            # post-accumulate hook AND the engine's grad-ready hook can both fire for a
            # parameter whose gradient one path writes directly): counted once, or the bucket
            # would launch before its last member is written
            return None
        self.ready.add(id(p))
        b = self.bucket_of[id(p)]
        self.pending[b] -= 1
        if self.pending[b] == 0:
            # nothing in the graph reads the averaged bucket: under capture (RCCL) the
            # all-reduce can become a node on a side branch of the backward graph
            act = graphs.detached(lambda: self._launch(b), capturable=self.use_avg)
            if defer:
                return act
            rec = graphs.active()
            if rec is not None:
                rec.cut([act])
                return None
            self._launch(b)
        return None

    def _launch(self, b):
        """Launch bucket b's all-reduce.  Inside a HIP-graph capture (graphs.Recorder in
        "capture" mode) the collective is recorded into the graph on a side branch: returns
        the joiner the recorder calls where the branch rejoins (wait + bf16 wire copy-back,
        both captured); every replay then runs it, and ``finish`` leaves the bucket alone."""
        if self.works[b] is not None:
            return None
        s, e, _ = self.buckets[b]
        view = self.flat.grad[s:e]
        if self.wire is not None:
            buf = self.wire[s:e]
            buf.copy_(view)
        else:
            buf = view
        # (one rank: the average IS the sum -- RCCL's single-rank PreMulSum would run a whole
        # extra pass over the bucket, a world-1 artifact that a ring all-reduce at N > 1 does
        # not have: profiles/r4/kstats_bs128_{plain,ddp}.txt)
        op = dist.ReduceOp.AVG if (self.use_avg and self.ws > 1) else dist.ReduceOp.SUM
        capturing = torch.cuda.is_available() and torch.cuda.is_current_stream_capturing()
        rec = graphs.active() if capturing else None
        if rec is not None and rec.checking:
            # in-graph collective check (graphs.py): snapshot the bucket in stream order right
            # before its captured all-reduce; compared with an eager all-reduce after replay
            def fix(ref, s=s, e=e, buf=buf):
                buf.copy_(ref)
                if self.wire is not None:
                    self.flat.grad[s:e].copy_(ref)
            rec.checks.append((buf.clone(), buf, op, self.pg, fix))
        work = dist.all_reduce(buf, op=op, group=self.pg, async_op=True)
        if capturing:
            self.in_graph.add(b)

            def join(w=work, s=s, e=e, buf=buf):
                w.wait()
                if graphs.CORRUPT_FOR_TEST:
                    buf.add_(1.0)  # (test hook: a broken in-graph collective)
                if self.wire is not None:
                    self.flat.grad[s:e].copy_(self.wire[s:e])
            return join
        self.works[b] = work
        self.cast[b] = self.wire is not None
        return None

    def finish(self):
        """Complete the gradient all-reduce (call once after backward).  Buckets whose
        all-reduce is part of the replayed backward graph are complete when the graph is; in
        a step where every hook fired inside a replay (no eager launch at all) they are
        skipped, any other bucket not launched yet (unused parameters) is launched now."""
        eager = any(w is not None for w in self.works)
        for b in range(len(self.buckets)):
            if self.works[b] is None and (eager or b not in self.in_graph):
                self._launch(b)
        for b, w in enumerate(self.works):
            if w is None:
                continue
            w.wait()
            s, e, _ = self.buckets[b]
            if self.cast[b]:
                self.flat.grad[s:e].copy_(self.wire[s:e])
                self.cast[b] = False
            if not self.use_avg and self.ws > 1:
                self.flat.grad[s:e].div_(self.ws)
        self.works = [None] * len(self.buckets)
        self.pending = [len(idx) for (_, _, idx) in self.buckets]
        self.ready = set()

    # ------------------------------------------------------------------ sync
    @torch.no_grad()
    def broadcast_parameters(self, src: int = 0):
        """X2: one broadcast of the whole flat parameter buffer (+ buffers)."""
        dist.broadcast(self.flat.data, src, group=self.pg)
        self.flat.refresh_shadow()
        self.sync_buffers(src)

    @torch.no_grad()
    def sync_buffers(self, src: int = 0):
        """X3: broadcast BatchNorm running statistics (DDP's broadcast_buffers)."""
        from .dist import broadcast_buffers
        broadcast_buffers(self.module, src, self.pg)

    def remove(self):
        for h in self._hooks:
            h.remove()
        self._hooks = []

    @property
    def bucket_sizes_mb(self):
        return [(e - s) * 4 / 2**20 for (s, e, _) in self.buckets]
