"""Fully-sharded data parallel over the flat parameter buffer (survey P6, X5).

The reference wraps the Transformer in torch-1.11 FSDP with CPU offload
(``transformer_test.py:387-392``): one flat parameter (auto-wrap never triggers at
29.3M params), all-gather of the full parameter for forward/backward, reduce-scatter of
the gradient, and — because NGD then sees a flat 1-D CPU shard — NGD preconditions the
wrong thing (survey Q17).

MI355X design (``FlatShardedDP``):

* the flat buffer is partitioned into ``world`` contiguous runs of WHOLE parameters
  (balanced by element count); rank r owns run r: its gradients after reduction, its
  optimizer state (MADGRAD/NGD/...), and its update;
* after backward one ``reduce_scatter_tensor`` (RCCL) delivers each rank the averaged
  gradient of its run (runs padded to equal length in a staging buffer so the
  collective is a single equal-chunk call); after the optimizer step one
  ``all_gather_into_tensor`` rebuilds the full parameters on every rank;
* NGD sees whole, correctly shaped parameters (Q17 fixed);
* gradient-norm clipping reduces the per-shard sum of squares across ranks (device
  scalar all-reduce, no host sync);
* with 288 GB of HBM per MI355X the full parameter copy stays resident between steps
  (ResNet-50: 94 MB): the communication schedule is FSDP's (reduce-scatter +
  all-gather = the same bytes as one all-reduce), optimizer state and gradient
  ownership are sharded 1/world; ``offload_optimizer=True`` keeps the owned optimizer
  state in pinned host memory (the reference's CPUOffload analogue).
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from ..utils.flat import ALIGN, FlatParams


def partition_slots(slots, world):
    """Contiguous partition of the flat slot list into ``world`` runs of whole
    parameters with balanced element counts (boundary placed nearest to
    total*r/world).  Runs may be empty when one parameter dominates."""
    sizes = [s.numel for s in slots]
    total = sum(sizes)
    cuts, acc, j = [0], 0, 0
    for r in range(1, world):
        target = total * r / world
        while j < len(slots) and acc + sizes[j] / 2 < target:
            acc += sizes[j]
            j += 1
        cuts.append(max(j, cuts[-1]))
    cuts.append(len(slots))
    return [(cuts[i], cuts[i + 1]) for i in range(world)]


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
        self.slots = []
        from ..utils.flat import Slot
        for s in slots:
            self.slots.append(Slot(s.name, s.param, s.offset - lo, s.numel, s.shape))
        self._by_param = {id(s.param): s for s in self.slots}

    @property
    def params(self):
        return [s.param for s in self.slots]

    def slot_of(self, p):
        return self._by_param[id(p)]

    def zero_grad(self):
        self.parent.zero_grad()

    def refresh_shadow(self):
        if self.shadow is not None:
            self.shadow.copy_(self.data)


class FlatShardedDP:
    def __init__(self, flat: FlatParams, module=None, process_group=None, broadcast_init=True):
        self.flat = flat
        self.module = module
        self.pg = process_group
        self.ws = dist.get_world_size(process_group)
        self.rank = dist.get_rank(process_group)
        self.use_avg = dist.get_backend(process_group) == "nccl"
        runs = partition_slots(flat.slots, self.ws)
        self.ranges = []
        for a, b in runs:
            if a == b:
                lo = hi = flat.numel
            else:
                lo = flat.slots[a].offset
                last = flat.slots[b - 1]
                hi = min((last.offset + last.numel + ALIGN - 1) // ALIGN * ALIGN, flat.numel)
            self.ranges.append((lo, hi))
        # slots are contiguous and 64-aligned, so consecutive non-empty runs already tile
        # the buffer; the trailing padding goes to the last non-empty run
        last_nonempty = max(r for r in range(self.ws) if self.ranges[r][0] < flat.numel)
        self.ranges[last_nonempty] = (self.ranges[last_nonempty][0], flat.numel)
        self.chunk = max(hi - lo for lo, hi in self.ranges)
        self.chunk = (self.chunk + ALIGN - 1) // ALIGN * ALIGN
        self.stage = torch.zeros(self.ws * self.chunk, device=flat.device, dtype=torch.float32)
        self.local = torch.zeros(self.chunk, device=flat.device, dtype=torch.float32)
        lo, hi = self.ranges[self.rank]
        a, b = runs[self.rank]
        self.view = ShardView(flat, lo, hi, flat.slots[a:b])
        if broadcast_init:
            dist.broadcast(flat.data, 0, group=self.pg)
            flat.refresh_shadow()

    def _pack(self, src: torch.Tensor):
        for r, (lo, hi) in enumerate(self.ranges):
            if hi > lo:
                self.stage[r * self.chunk:r * self.chunk + (hi - lo)].copy_(src[lo:hi])

    def _unpack(self, dst: torch.Tensor):
        for r, (lo, hi) in enumerate(self.ranges):
            if hi > lo:
                dst[lo:hi].copy_(self.stage[r * self.chunk:r * self.chunk + (hi - lo)])

    def finish_backward(self):
        """Reduce-scatter: rank r receives the averaged gradient of run r."""
        self._pack(self.flat.grad)
        op = dist.ReduceOp.AVG if self.use_avg else dist.ReduceOp.SUM
        dist.reduce_scatter_tensor(self.local, self.stage, op=op, group=self.pg)
        if not self.use_avg:
            self.local.div_(self.ws)
        lo, hi = self.ranges[self.rank]
        self.flat.grad[lo:hi].copy_(self.local[:hi - lo])

    def after_step(self):
        """All-gather the updated runs into every rank's full parameter buffer."""
        lo, hi = self.ranges[self.rank]
        self.local.zero_()
        self.local[:hi - lo].copy_(self.flat.data[lo:hi])
        dist.all_gather_into_tensor(self.stage, self.local, group=self.pg)
        with torch.no_grad():
            self._unpack(self.flat.data)
        self.flat.refresh_shadow()
        # gradients outside the owned run were consumed by the reduce-scatter
        self.flat.grad.zero_()
