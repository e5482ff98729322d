"""Sharded-optimizer data parallel for NGD: every rank holds the full parameters, the
gradient all-reduce overlaps backward bucket by bucket, and rank r preconditions + updates
only the parameters it owns; the updated parameters are then all-gathered.

Used for the reference's distributed NGD run (``run_distributed.sh:2``: ``--distributed
--ngd``; ``ngd_optimizer.py:452-508``, DDP reducer overlap ``resnet50_test.py:716``): under
plain DDP every rank would precondition every parameter -- identical work repeated
``world`` times (ResNet-50 NGD update step ~8.6 ms, a non-update step ~2.9 ms, against
~5.6 ms of compute per step at 8 GPUs).  Here each rank owns whole parameters (NGD
preconditions along every axis of a parameter, so ownership is per parameter, not per flat
chunk), balanced by NGD cost (``utils/flat.ngd_balanced_order``), and keeps NGD state (W,
d, rho per axis) only for those: the NGD cost per rank is ~1/world and the result equals
single-process NGD on the averaged gradient.

Communication, MI355X-first:

* **gradients** live in a second flat buffer in *backward order* (``grad_space``), so the
  DDP bucket reducer (``parallel/ddp.py``) all-reduces each bucket from the gradient-ready
  hooks while backward continues -- and, when the engine's backward is captured as HIP
  graphs, between the replayed segments (``parallel/graphs.py``).  Why an all-reduce and
  not a per-bucket reduce-scatter: ownership is whole parameters, and a reduce-scatter
  needs ``world`` EQUAL chunks per bucket; ResNet-50's 4-9 MB stage-5 weights would pad an
  8-way bucket split ~3x.  The all-reduce moves 2x the bytes of a reduce-scatter but all of
  it overlaps backward, where the old post-backward reduce-scatter was fully exposed.
* the rank's owned gradients are gathered from the averaged buffer into its optimizer view
  (1/world of the bytes, multi-tensor copy) -- the view IS run r of the partitioned
  parameter buffer's twin gradient, so the optimizer kernels see one contiguous range;
* **parameters** stay in the partitioned layout (``FlatParams(partition=world)``: run r at
  offset r*chunk), so the post-step all-gather is ONE in-place
  ``all_gather_into_tensor`` on RCCL (the rank's run is already at its slot of the output:
  no staging copy).
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from ..utils.flat import ALIGN, FlatParams, Slot


class ShardView:
    """FlatParams-compatible view of one rank's run (what the optimizer updates)."""

    def __init__(self, flat: FlatParams, lo: int, hi: int, slots):
        self.parent = flat
        self.lo, self.hi = lo, hi
        self.numel = hi - lo
        self.data = flat.data[lo:hi]
        self.grad = flat.grad[lo:hi]
        self.shadow = flat.shadow[lo:hi] if flat.shadow is not None else None
        self.device = flat.device
        self.slots = [Slot(s.name, s.param, s.offset - lo, s.numel, s.shape) for s in slots]
        self._by_param = {id(s.param): s for s in self.slots}

    @property
    def params(self):
        return [s.param for s in self.slots]

    def slot_of(self, p):
        return self._by_param[id(p)]

    def zero_grad(self):
        self.grad.zero_()

    def refresh_shadow(self):
        if self.shadow is not None:
            self.shadow.copy_(self.data)


class GradSpace:
    """Backward-ordered flat gradient buffer (what the bucket reducer all-reduces): every
    ``p.grad`` is a view into it; slots in model-reversed order so buckets fill in backward
    order (the ``FlatParams`` non-partitioned layout)."""

    def __init__(self, params_in_backward_order, device, dtype):
        self.slots, off = [], 0
        for n, p in params_in_backward_order:
            self.slots.append(Slot(n, p, off, p.numel(), p.shape))
            off += (p.numel() + ALIGN - 1) // ALIGN * ALIGN
        self.numel = off
        self.device = torch.device(device)
        self.grad = torch.zeros(self.numel, device=self.device, dtype=dtype)
        self.data = None  # (the reducer only broadcasts parameters when asked to)
        self._by_param = {id(s.param): s for s in self.slots}
        self.bind()

    def bind(self):
        for s in self.slots:
            s.param.grad = self.grad[s.offset:s.offset + s.numel].view(s.shape)

    def slot_of(self, p):
        return self._by_param[id(p)]

    def refresh_shadow(self):
        pass


class ShardedOptimizerDP:
    """Bucketed all-reduce overlapped with backward + per-rank optimizer + all-gather.

    ``flat`` must be built with ``partition=world`` (see module docstring).  ``finish_backward``
    lands the averaged gradients of the rank's parameters in ``view.grad``; ``after_step``
    all-gathers the updated runs."""

    sharded_optimizer = True

    def __init__(self, flat: FlatParams, module=None, process_group=None, broadcast_init=True, bucket_mb=25.0,
                 first_bucket_mb=1.0, comm_dtype=None):
        from .ddp import BucketReducer
        self.flat = flat
        self.module = module
        self.pg = process_group
        self.ws = dist.get_world_size(process_group)
        self.rank = dist.get_rank(process_group)
        if flat.runs is None or len(flat.runs) != self.ws:
            raise ValueError("ShardedOptimizerDP needs FlatParams(partition=world_size)")
        self.nccl = dist.get_backend(process_group) == "nccl"
        c = flat.chunk
        self.lo, self.hi = self.rank * c, (self.rank + 1) * c
        a, b = flat.runs[self.rank]
        self.view = ShardView(flat, self.lo, self.hi, flat.slots[a:b])
        # backward order = reversed module registration order (FlatParams' default layout)
        if module is not None:
            named = [(n, p) for n, p in module.named_parameters() if p.requires_grad]
            known = {id(s.param) for s in flat.slots}
            named = [(n, p) for n, p in named if id(p) in known]
            have = {id(p) for _, p in named}
            named += [(s.name, s.param) for s in flat.slots if id(s.param) not in have]
            named = named[::-1]
        else:
            named = [(s.name, s.param) for s in flat.slots]
        self.grad_space = GradSpace(named, flat.device, flat.grad.dtype)
        if broadcast_init:
            dist.broadcast(flat.data, 0, group=self.pg)
            flat.refresh_shadow()
        self.reducer = BucketReducer(self.grad_space, module, process_group, bucket_mb=bucket_mb,
                                     first_bucket_mb=first_bucket_mb, comm_dtype=comm_dtype, broadcast_init=False)
        # owned gradient views (source: averaged backward-ordered buffer, destination: the
        # optimizer's contiguous run)
        gs = self.grad_space
        self._src = [gs.grad[gs.slot_of(s.param).offset:gs.slot_of(s.param).offset + s.numel] for s in self.view.slots]
        self._dst = [self.view.grad[s.offset:s.offset + s.numel] for s in self.view.slots]
        # gloo cannot all-gather in place: stage the run (RCCL: the run is already at its
        # slot of the output buffer)
        self.local = None if self.nccl else torch.empty(c, device=flat.device, dtype=flat.data.dtype)

    @property
    def buckets(self):
        return self.reducer.buckets

    def finish_backward(self):
        """Wait for the overlapped bucket all-reduces; the averaged gradients of the rank's
        own parameters go to the optimizer view."""
        self.reducer.finish()
        if self._dst:
            torch._foreach_copy_(self._dst, self._src)

    def after_step(self):
        """All-gather every rank's updated run into the full parameter buffer; clear the
        backward-ordered gradient for the next accumulation (the optimizer cleared its run).
        The clear runs on the compute stream WHILE the all-gather runs on RCCL's stream (the
        gather is issued async and joined after): the ~100 MB memset leaves the critical path.
        (It cannot be dropped: the engine's 1x1 weight gradients accumulate with split-K
        atomics, so every step starts from a zeroed buffer.)"""
        work = None
        if self.ws > 1:
            if self.local is None:
                work = dist.all_gather_into_tensor(self.flat.data, self.view.data, group=self.pg, async_op=True)
            else:
                self.local.copy_(self.view.data)
                work = dist.all_gather_into_tensor(self.flat.data, self.local, group=self.pg, async_op=True)
        self.grad_space.grad.zero_()
        if work is not None:
            work.wait()
        self.flat.refresh_shadow()

    def sync_buffers(self, src: int = 0):
        from .dist import broadcast_buffers
        broadcast_buffers(self.module, src, self.pg)
