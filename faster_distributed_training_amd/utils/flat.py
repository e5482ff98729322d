"""Flat parameter / gradient storage.

All trainable parameters of a model are re-homed into ONE contiguous fp32 buffer
(``FlatParams.data``) and their gradients into another (``FlatParams.grad``); every
``p.data`` / ``p.grad`` becomes a view.  Consequences on MI355X:

* optimizers (``optim/``), gradient clipping and AMP unscale are single fused HIP
  launches over the whole model (23.5M elements for ResNet-50) instead of
  69 tensors x several ops;
* the DDP reducer's buckets are contiguous slices of ``grad`` (gradient-as-bucket-view,
  no flatten/unflatten copies), laid out in *reverse* registration order so they fill
  in backward order;
* FSDP shards and checkpoint I/O are slices of the same buffer;
* an optional bf16 shadow copy (``shadow``) is rewritten by the optimizer kernel itself
  so compute kernels read bf16 weights without a per-step cast pass.

``p.grad`` must never be replaced (no ``zero_grad(set_to_none=True)``): use
``FlatParams.zero_grad()``; autograd then accumulates in place into the views.
"""
from __future__ import annotations

from dataclasses import dataclass

import math

import os

import torch
import torch.nn as nn

ALIGN = 64  # elements; keeps every view 256-B aligned for 16-B vector access


@dataclass
class Slot:
    name: str
    param: nn.Parameter
    offset: int
    numel: int
    shape: torch.Size


def _aligned(n: int) -> int:
    return (n + ALIGN - 1) // ALIGN * ALIGN


def partition_runs(sizes, world):
    """Contiguous partition of a list of sizes into ``world`` runs with balanced totals
    (each boundary placed nearest to total*r/world).  Returns [(first, last+1)] per run;
    runs may be empty when one item dominates."""
    total = sum(sizes)
    cuts, acc, j = [0], 0, 0
    for r in range(1, world):
        target = total * r / world
        while j < len(sizes) and acc + sizes[j] / 2 < target:
            acc += sizes[j]
            j += 1
        cuts.append(max(j, cuts[-1]))
    cuts.append(len(sizes))
    return [(cuts[i], cuts[i + 1]) for i in range(world)]


# NGD cost of a parameter in element-equivalents: each preconditioned axis (dim > 1) costs a
# fixed ~25 us of launches and small-matrix math whatever its size (measured: ResNet-50 NGD
# with an element-balanced 8-way split ran 1.7 ms on the rank holding the stem + stage 1
# -- dozens of small tensors -- and 0.3-0.5 ms on the others, scripts/bench_ngd.py --world)
# Round 6: 200000 -> 400000 from a sweep of every simulated world-8 rank on one box, back to back
# (bench.py --simulate-world 8, profiles/r6/sim/balance/axis_cost_sweep.txt): slowest rank of
# ResNet-50 NGD + meta-mixup 7.23 / 7.46 -> 7.19 / 7.14 ms, of the transformer at B=32 4.52 ->
# 4.39 ms (the per-axis fixed cost -- launches, small-matrix math -- was underweighted: the rank
# holding the most shape groups was the slowest)
NGD_AXIS_COST = int(os.environ.get("FDT_NGD_AXIS_COST", "400000"))
NGD_SLACK = float(os.environ.get("FDT_NGD_SLACK", "1.15"))


def ngd_cost(shape) -> int:
    n = 1
    for d in shape:
        n *= d
    return n + NGD_AXIS_COST * sum(1 for d in shape if d > 1)


def ngd_balanced_order(shapes, world, slack=None):
    """Order of parameters (indices into ``shapes``) such that cutting it into ``world``
    contiguous runs balances the NGD cost per rank while every run stays within
    ``slack`` x the even share of elements (the flat chunk, hence the reduce-scatter /
    all-gather size, is the largest run).  Greedy: largest cost first onto the cheapest
    rank with element room.  Returns (order, runs)."""
    slack = NGD_SLACK if slack is None else slack
    sizes = [_aligned(math.prod(sh)) for sh in shapes]
    cap = max(max(sizes, default=0), int(slack * sum(sizes) / max(world, 1)) + ALIGN)
    cost, elems = [0] * world, [0] * world
    members = [[] for _ in range(world)]
    for i in sorted(range(len(shapes)), key=lambda i: -ngd_cost(shapes[i])):
        fits = [r for r in range(world) if elems[r] + sizes[i] <= cap]
        r = min(fits, key=lambda r: (cost[r], elems[r])) if fits else min(range(world), key=lambda r: elems[r])
        members[r].append(i)
        cost[r] += ngd_cost(shapes[i])
        elems[r] += sizes[i]
    order, runs = [], []
    for r in range(world):
        a = len(order)
        order += sorted(members[r])  # keep model order inside a run
        runs.append((a, len(order)))
    return order, runs


def _adjacent_groups(named, groups):
    """Reorder (name, param) so that each group's parameters (a list, in the given order) sit
    next to each other where the group's first member was: e.g. the Q / K / V projections of
    an attention block, whose stacked bf16 weights the fused projection can then read as ONE
    contiguous view of the shadow buffer instead of concatenating them every forward
    (ops/linear.py ``_LinearCat``)."""
    pos = {id(p): i for i, (_, p) in enumerate(named)}
    moved = {}
    for grp in groups:
        idx = [pos.get(id(p)) for p in grp]
        if len(grp) < 2 or any(i is None for i in idx) or any(id(p) in moved for p in grp):
            continue
        first = min(idx)
        for p in grp:
            moved[id(p)] = first
    if not moved:
        return named
    out, placed = [], set()
    by_first = {}
    for grp in groups:
        if grp and id(grp[0]) in moved:
            by_first.setdefault(moved[id(grp[0])], []).append(grp)
    for i, (n, p) in enumerate(named):
        for grp in by_first.get(i, []):
            for q in grp:
                out.append(named[pos[id(q)]])
                placed.add(id(q))
        if id(p) not in moved and id(p) not in placed:
            out.append((n, p))
    return out


class FlatParams:
    """``partition=W``: the slots are split into W contiguous runs of whole parameters
    (balanced) and run r is placed at offset r*chunk (chunk = the longest run, aligned), so
    the buffers are W equal chunks: reduce-scatter / all-gather need no packing (the
    sharded-optimizer data parallel of ``parallel/zero.py``).  ``balance="ngd"``: runs
    balance the NGD preconditioning cost (``ngd_balanced_order``; parameters are regrouped,
    not kept in model order) instead of the element count alone."""

    def __init__(self, module_or_params, device=None, reverse=True, with_shadow=False, names=None, partition=0,
                 dtype=torch.float32, balance="numel", adjacent="shape"):
        if isinstance(module_or_params, nn.Module):
            named = [(n, p) for n, p in module_or_params.named_parameters() if p.requires_grad]
        else:
            plist = list(module_or_params)
            named = [(names[i] if names else f"p{i}", p) for i, p in enumerate(plist)]
        if reverse:
            named = named[::-1]
        # adjacent: "shape" = every same-shape parameter of the model in one run (single GPU: NGD's
        # shape groups become views), "layer" = only one block's Q / K / V (data-parallel
        # world > 1: whole-model shape runs would park every layer's weights in the first
        # gradient buckets, which then wait for layer 0's backward -- no comm / backward
        # overlap), None / FDT_FLAT_ADJACENT=0 = registration order
        if (adjacent and isinstance(module_or_params, nn.Module) and hasattr(module_or_params, "flat_adjacent")
                and os.environ.get("FDT_FLAT_ADJACENT", "1") != "0"):
            named = _adjacent_groups(named, module_or_params.flat_adjacent(adjacent))
        self.slots: list[Slot] = []
        self.runs = None
        self.chunk = 0
        if partition and partition >= 1:  # (partition=1: one run, the world-size-1 case)
            if balance == "ngd" and partition > 1:
                order, self.runs = ngd_balanced_order([tuple(p.shape) for _, p in named], partition)
                named = [named[i] for i in order]
            else:
                self.runs = partition_runs([_aligned(p.numel()) for _, p in named], partition)
            self.chunk = max(sum(_aligned(named[i][1].numel()) for i in range(a, b)) for a, b in self.runs)
            self.chunk = max(self.chunk, ALIGN)
            for r, (a, b) in enumerate(self.runs):
                off = r * self.chunk
                for n, p in named[a:b]:
                    self.slots.append(Slot(n, p, off, p.numel(), p.shape))
                    off += _aligned(p.numel())
            self.numel = partition * self.chunk
        else:
            off = 0
            for n, p in named:
                k = p.numel()
                self.slots.append(Slot(n, p, off, k, p.shape))
                off += _aligned(k)
            self.numel = off
        dev = device if device is not None else (named[0][1].device if named else torch.device("cpu"))
        self.device = torch.device(dev)
        # (dtype: fp32 master weights; fp64 for CPU golden tests)
        self.data = torch.zeros(self.numel, device=self.device, dtype=dtype)
        self.grad = torch.zeros(self.numel, device=self.device, dtype=dtype)
        self.shadow = torch.zeros(self.numel, device=self.device, dtype=torch.bfloat16) if with_shadow else None
        with torch.no_grad():
            for s in self.slots:
                v = self.data[s.offset:s.offset + s.numel].view(s.shape)
                v.copy_(s.param.data.to(self.device, dtype))
                s.param.data = v
                s.param.grad = self.grad[s.offset:s.offset + s.numel].view(s.shape)
        self.refresh_shadow()
        self._by_param = {id(s.param): s for s in self.slots}

    # ------------------------------------------------------------------ helpers
    @property
    def params(self):
        return [s.param for s in self.slots]

    def slot_of(self, p) -> Slot:
        return self._by_param[id(p)]

    def grad_view(self, p):
        s = self.slot_of(p)
        return self.grad[s.offset:s.offset + s.numel].view(s.shape)

    def shadow_view(self, p):
        if self.shadow is None:
            return None
        s = self.slot_of(p)
        return self.shadow[s.offset:s.offset + s.numel].view(s.shape)

    def zero_grad(self):
        self.grad.zero_()
        self.rebind_grads()

    def rebind_grads(self):
        """Re-attach grad views if something replaced ``p.grad`` (e.g. a foreign
        ``zero_grad(set_to_none=True)``)."""
        for s in self.slots:
            g = s.param.grad
            want = self.grad[s.offset:s.offset + s.numel]
            if g is None or g.data_ptr() != want.data_ptr():
                if g is not None:
                    want.view(s.shape).copy_(g)
                s.param.grad = want.view(s.shape)

    # a module whose native engine keeps packed copies of the weights (ops/resnet_fused.py Plan):
    # the optimizer writes them in its fused step; out-of-band weight writes must drop that claim
    pack_owner = None

    def invalidate_packed(self):
        plan = getattr(self.pack_owner, "_plan", None)
        if plan is not None:
            plan.invalidate_pack()

    def refresh_shadow(self):
        self.invalidate_packed()
        if self.shadow is not None:
            with torch.no_grad():
                self.shadow.copy_(self.data)

    def load_from_params(self):
        """Re-sync after params were assigned new storage (e.g. load_state_dict on a
        module whose params were replaced)."""
        with torch.no_grad():
            for s in self.slots:
                if s.param.data.data_ptr() != self.data[s.offset:].data_ptr():
                    self.data[s.offset:s.offset + s.numel].copy_(s.param.data.reshape(-1))
                    s.param.data = self.data[s.offset:s.offset + s.numel].view(s.shape)
        self.refresh_shadow()
