"""Sharded-optimizer data parallel (ZeRO-2 style): every rank holds the full parameters,
gradients are reduce-scattered so rank r receives the averaged gradient of ITS parameters
only, rank r runs the optimizer on those, and the updated parameters are all-gathered.

Used for the reference's distributed NGD run (``run_distributed.sh:2``: ``--distributed
--ngd``; ``ngd_optimizer.py:452-508``): under plain DDP every rank would precondition every
parameter -- identical work repeated ``world`` times (ResNet-50 NGD update step ~10 ms, a
non-update step ~4 ms, against ~1 ms of compute per step at 8 GPUs).  Here each rank owns
whole parameters (NGD preconditions along every axis of a parameter, so ownership is per
parameter, not per flat chunk), balanced by element count, and keeps NGD state (W, d, rho
per axis) only for those: the NGD cost per rank is ~1/world, and the result equals
single-process NGD on the averaged gradient.

Layout: the flat buffers are built with ``FlatParams(partition=world)``, which places run r
at offset r*chunk -- the gradient buffer IS the reduce-scatter input and the parameter
buffer the all-gather output, no packing.  Communication = one reduce-scatter + one
all-gather of the flat buffer (the bytes of one all-reduce).
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from ..utils.flat import FlatParams, Slot


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


class ShardedOptimizerDP:
    """Reduce-scatter gradients / all-gather parameters around a per-rank optimizer.

    ``flat`` must be built with ``partition=world`` (see module docstring)."""

    sharded_optimizer = True

    def __init__(self, flat: FlatParams, module=None, process_group=None, broadcast_init=True):
        self.flat = flat
        self.module = module
        self.pg = process_group
        self.ws = dist.get_world_size(process_group)
        self.rank = dist.get_rank(process_group)
        if flat.runs is None or len(flat.runs) != self.ws:
            raise ValueError("ShardedOptimizerDP needs FlatParams(partition=world_size)")
        self.use_avg = dist.get_backend(process_group) == "nccl"
        c = flat.chunk
        self.lo, self.hi = self.rank * c, (self.rank + 1) * c
        a, b = flat.runs[self.rank]
        self.view = ShardView(flat, self.lo, self.hi, flat.slots[a:b])
        self.local = torch.empty(c, device=flat.device, dtype=flat.data.dtype)
        if broadcast_init:
            dist.broadcast(flat.data, 0, group=self.pg)
            flat.refresh_shadow()

    def finish_backward(self):
        """Reduce-scatter: rank r receives the averaged gradient of its run."""
        op = dist.ReduceOp.AVG if self.use_avg else dist.ReduceOp.SUM
        dist.reduce_scatter_tensor(self.local, self.flat.grad, op=op, group=self.pg)
        if not self.use_avg:
            self.local.div_(self.ws)
        self.view.grad.copy_(self.local)

    def after_step(self):
        """All-gather every rank's updated run into the full parameter buffer."""
        self.local.copy_(self.view.data)
        dist.all_gather_into_tensor(self.flat.data, self.local, group=self.pg)
        self.flat.refresh_shadow()
        # the backward accumulates into the whole flat gradient: clear what the optimizer
        # (which zeroes only its own run) did not
        self.flat.grad.zero_()

    def sync_buffers(self, src: int = 0):
        from .dist import broadcast_buffers
        broadcast_buffers(self.module, src, self.pg)
