"""Fully-sharded data parallel (ZeRO-3): parameters sharded at rest, gathered per wrap unit.

Reference: ``transformer_test.py:387-392`` wraps the Transformer in torch-1.11 FSDP with
``size_based_auto_wrap_policy`` and ``CPUOffload(offload_params=True)`` (survey P6, X5; at
29.3M parameters the policy never fires, so the reference has ONE unit and NGD sees a flat
1-D CPU shard -- survey Q17).  BASELINE.json config 5 asks for ResNet-50 FSDP full-shard.

MI355X design (``FullyShardedDP``):

* **wrap units**: ResNet: stem, conv2_x .. conv5_x, fc; Transformer: the embeddings, every
  attention / FFN sublayer, pooler + classifier (``default_units``); or a size-based policy
  (``min_params``), like the reference's ``size_based_auto_wrap_policy``.  Parameters
  outside every unit form a root unit that stays gathered.
* **at rest** each rank keeps only its shard of every unit: the fp32 master copy, its
  gradient and the optimizer state over it (``self.space``: a FlatParams-like object the
  fused optimizers and the gradient clipper run on).  Full unit parameters exist only while
  the unit is in use: the storage behind the parameter views is resized to 0 in between.
* **layout**: a unit's full buffer is ``world`` equal chunks, chunk r = rank r's shard, so
  one ``all_gather_into_tensor`` rebuilds it and one ``reduce_scatter_tensor`` of the unit's
  gradient buffer delivers every rank its averaged shard (RCCL, no packing).  Shard mode
  ``flat`` cuts the unit's parameters evenly (elementwise optimizers); mode ``param`` gives
  every rank whole parameters (NGD preconditions along parameter axes -- Q17: it sees
  correctly shaped tensors, never a flat shard).
* **schedule**: forward: a unit waits for its all-gather and immediately launches the
  next unit's (prefetch), runs, then frees its parameters; backward (entered through a hook
  on the unit's output gradient): gather again + prefetch the previous unit, gradients
  accumulate into a unit gradient buffer, and when the unit's last gradient is final
  (post-accumulate hooks) its reduce-scatter is launched asynchronously while backward
  continues; ``finish_backward`` only waits.  The optimizer then updates the shards; the
  next forward gathers the new values -- no post-step all-gather.
* **offload**: ``offload=True`` keeps shards (and optimizer state) in pinned host memory
  like the reference's ``CPUOffload``: gathers copy the shard H2D first, gradients come back
  D2H after the reduce-scatter, and the optimizer runs on the host (``offload_optimizer=
  "host"``, the faithful mode).  ``offload_optimizer="device"``: the parameter shards still
  live in pinned host memory between steps (every gather stages them H2D; after each step the
  updated shard is mirrored back D2H on the copy stream, ahead of the next step's gathers on
  that same stream), but the optimizer -- NGD / MADGRAD math and state -- runs on the GPU over
  the device staging copies, and the averaged gradient never leaves the device.
* the fused ResNet engine (one autograd node for the whole body) drives its units itself at
  stage boundaries (``pre_forward`` / ``post_forward`` / ``pre_backward`` / ``post_backward``,
  ``ops/resnet_fused.py``) and packs / releases its bf16 weight layouts per stage.
* **static mode** (``static=True``, the engine's HIP-graph path): every unit keeps its
  gathered-parameter and gradient buffers for the whole run (fixed addresses, so the body can
  be captured as graphs) -- FSDP's SHARD_GRAD_OP schedule: parameters are gathered once per
  step in forward (next unit prefetched) and reused by backward, gradients are reduce-
  scattered per unit from backward, the optimizer state and master weights stay sharded.
  While a capture is recording, each collective becomes an action between two graph
  segments (``parallel/graphs.Recorder.cut``): a replay waits for unit i's all-gather and
  launches unit i+1's before replaying stage i, and launches unit i's reduce-scatter right
  after stage i's backward segment -- communication keeps overlapping compute.

Memory: with 288 GB per MI355X this is a capability, not a necessity, for these models;
``peak_full_bytes`` reports the largest amount of gathered parameter + unit-gradient storage
alive at once.  The schedule bounds it by max_i(2 b_i + b_(i-1) + b_(i+1)) + 2 b_root (unit
i gathered with its gradient buffer, unit i-1 prefetched, unit i+1's reduce-scatter in
flight; b = a unit's full fp32 bytes).
"""
from __future__ import annotations

import contextlib

import torch
import torch.distributed as dist
import torch.nn as nn

from ..utils.flat import ALIGN, Slot, partition_runs


def _al(n):
    return (n + ALIGN - 1) // ALIGN * ALIGN


def default_units(model: nn.Module):
    """Wrap units for the models of this package (name, module) in forward order."""
    names = dict(model.named_children())
    if all(k in names for k in ("conv1", "conv2_x", "conv3_x", "conv4_x", "conv5_x", "fc")):
        return [(k, names[k]) for k in ("conv1", "conv2_x", "conv3_x", "conv4_x", "conv5_x", "fc")]
    if "sublayer_attention" in names and "sublayer_ffn" in names:
        units = [("input_embeddings", model.input_embeddings)]
        for i, (a, f) in enumerate(zip(model.sublayer_attention, model.sublayer_ffn)):
            units += [(f"sublayer_attention.{i}", a), (f"sublayer_ffn.{i}", f)]
        units += [("pooler", model.pooler), ("classifier", model.classifier)]
        return units
    return size_based_units(model, 10**6)


def size_based_units(model: nn.Module, min_params: int):
    """Reference-style size-based auto wrap: a maximal submodule with >= min_params
    parameters becomes a unit (recursively, children first)."""
    out = []

    def visit(prefix, mod):
        n = sum(p.numel() for p in mod.parameters())
        big_children = False
        for name, ch in mod.named_children():
            if sum(p.numel() for p in ch.parameters()) >= min_params:
                big_children = True
        if big_children:
            for name, ch in mod.named_children():
                visit(f"{prefix}{name}.", ch)
        elif n >= min_params and prefix:
            out.append((prefix[:-1], mod))

    visit("", model)
    return out


class SpaceView:
    """The rank's shard space seen by the optimizer / clipper (FlatParams interface)."""

    def __init__(self, data, grad, slots, device):
        self.data, self.grad = data, grad
        self.numel = data.numel()
        self.slots = slots
        self.shadow = None
        self.device = device
        self._by_param = {id(s.param): s for s in slots}

    @property
    def params(self):
        return [s.param for s in self.slots]

    def slot_of(self, p):
        return self._by_param[id(p)]

    def zero_grad(self):
        self.grad.zero_()

    def refresh_shadow(self):
        pass


class Unit:
    def __init__(self, fs, idx, name, params, mode, root=False):
        self.fs, self.idx, self.name, self.root = fs, idx, name, root
        self.params = params  # [(qualified name, Parameter)]
        ws, rank = fs.ws, fs.rank
        sizes = [_al(p.numel()) for _, p in params]
        if mode == "param":
            runs = partition_runs(sizes, ws)
            self.chunk = max(ALIGN, max(sum(sizes[a:b]) for a, b in runs))
            self.pos = {}
            for r, (a, b) in enumerate(runs):
                off = r * self.chunk
                for i in range(a, b):
                    self.pos[i] = off
                    off += sizes[i]
            mine = runs[rank]
            self.owned = [(i, self.pos[i] - rank * self.chunk) for i in range(mine[0], mine[1])]
        else:
            total = sum(sizes)
            self.chunk = _al(-(-total // ws))
            self.pos, off = {}, 0
            for i, s in enumerate(sizes):
                self.pos[i] = off
                off += s
            lo, hi = rank * self.chunk, (rank + 1) * self.chunk
            # whole parameters inside this rank's chunk (NGD-usable; flat mode is for
            # elementwise optimizers, the slots only name the parameters)
            self.owned = [(i, self.pos[i] - lo) for i in range(len(params))
                          if self.pos[i] >= lo and self.pos[i] + params[i][1].numel() <= hi]
        self.numel = ws * self.chunk
        self.slot = None  # full-shard static mode: index of the ring slot holding this unit
        dev = fs.device
        self.full = torch.zeros(self.numel, device=dev, dtype=torch.float32)
        # param_dtype bf16: the all-gather moves bf16 (half the bytes on xGMI) into this
        # buffer, upcast into ``full`` after the wait (FSDP MixedPrecision(param_dtype=bf16):
        # compute sees bf16-rounded weights, the sharded fp32 masters are what the optimizer
        # updates)
        self.full16 = (torch.zeros(self.numel, device=dev, dtype=fs.param_dtype)
                       if fs.param_dtype is not None else None)
        self.gfull = torch.zeros(self.numel, device=dev, dtype=torch.float32)
        self.views = []
        with torch.no_grad():
            for i, (n, p) in enumerate(params):
                v = self.full[self.pos[i]:self.pos[i] + p.numel()].view(p.shape)
                v.copy_(p.data)
                self.views.append(v)
                p.data = v
        self.gathered = True
        self.grads_live = False
        self.work = None      # pending all-gather
        self.rs_work = None   # pending reduce-scatter
        self.pending = 0      # gradients still to arrive in this backward
        self.bwd_started = False

    # ------------------------------------------------------------ storage
    def _bytes(self):
        return self.numel * 4

    def _alloc(self, t):
        st = t.untyped_storage()
        if st.size() == 0:
            st.resize_(self._bytes())

    def _free(self, t):
        if self.fs.static:
            return  # static mode: buffers keep their addresses (captured graphs read them)
        st = t.untyped_storage()
        if st.size() != 0:
            st.resize_(0)

    # ------------------------------------------------------------ gather / reshard
    def bind_ring(self, slot, full, full16, gfull):
        """Full-shard static mode: this unit's gathered parameters / gradient live in ring
        slot ``slot`` (fixed addresses shared with the other units of that slot)."""
        self.slot = slot
        self.full, self.full16, self.gfull = full[:self.numel], (None if full16 is None else full16[:self.numel]), \
            gfull[:self.numel]
        with torch.no_grad():
            for i, (n, p) in enumerate(self.params):
                v = self.full[self.pos[i]:self.pos[i] + p.numel()].view(p.shape)
                self.views[i] = v
                p.data = v
        self.gathered = False

    def _claim_slot(self):
        """Ring: take this unit's slot from its previous owner (whose parameters are about to
        be overwritten; an in-flight gather of theirs is ordered first)."""
        fs = self.fs
        owner = fs.slot_owner[self.slot]
        if owner is self:
            return
        if owner is not None:
            if owner.work is not None:
                owner.work.wait()
                owner.work = None
            owner.gathered = False
        fs.slot_owner[self.slot] = self
        self.gathered = False

    def gather(self, wait=True, exact=False):
        """All-gather this unit's parameters (``exact``: fp32 wire even with a bf16
        param_dtype -- checkpoint I/O)."""
        fs = self.fs
        if self.slot is not None:
            self._claim_slot()
        if not self.gathered and self.work is None:
            self._alloc(self.full)
            fs._account()
            lowp = self.full16 is not None and not exact
            self._lowp = lowp
            dst = self.full16 if lowp else self.full
            if fs.offload and fs.copy_stream is not None:
                # pinned-host shard -> device staging on the copy stream, and the all-gather
                # launched from that stream (RCCL orders after the copy): the compute stream
                # only meets this unit at its wait
                fs.copy_stream.wait_stream(torch.cuda.current_stream(fs.device))  # staging reuse
                with torch.cuda.stream(fs.copy_stream):
                    src = fs.shard_chunk(self, lowp)
                    self.work = dist.all_gather_into_tensor(dst, src, group=fs.pg, async_op=True)
            else:
                src = fs.shard_chunk(self, lowp)
                self.work = dist.all_gather_into_tensor(dst, src, group=fs.pg, async_op=True)
        if wait and self.work is not None:
            self.work.wait()
            self.work = None
            if getattr(self, "_lowp", False):
                self.full.copy_(self.full16)  # bf16 wire -> the fp32 views the modules read
            self.gathered = True

    def reshard(self):
        if self.root or not self.gathered or self.work is not None or self.fs.static:
            return
        self._free(self.full)
        self.gathered = False

    # ------------------------------------------------------------ backward
    def begin_backward(self, gather=True):
        if self.bwd_started:
            return
        self.bwd_started = True
        if gather:
            self.gather(wait=True)
        self._alloc(self.gfull)
        self.gfull.zero_()
        for i, (n, p) in enumerate(self.params):
            p.grad = self.gfull[self.pos[i]:self.pos[i] + p.numel()].view(p.shape)
        self.grads_live = True
        self.pending = sum(1 for _, p in self.params if p.requires_grad)
        self.fs._account()

    def grad_ready(self):
        self.pending -= 1
        if self.pending == 0:
            if self.fs.static:
                from . import graphs
                if graphs.active() is not None:
                    # backward being captured (module-hook units, e.g. the transformer's
                    # sublayers): the reduce-scatter is an action of every replay
                    self.grads_live = False

                    def act(u=self):
                        u.grads_live = True
                        u.reduce()
                    self.fs._deferred(graphs.detached(act))
                    return
            self.reduce()

    def reduce(self):
        """Launch the reduce-scatter of this unit's gradient (async), release buffers."""
        fs = self.fs
        if not self.grads_live or self.rs_work is not None:
            return
        if fs.static:
            # gradient views stay bound to the persistent buffer; only the collective
            op = dist.ReduceOp.AVG if (fs.use_avg and fs.ws > 1) else dist.ReduceOp.SUM  # (1 rank: sum)
            self.rs_work = dist.reduce_scatter_tensor(fs.grad_chunk(self), self.gfull, op=op, group=fs.pg,
                                                      async_op=True)
            self.grads_live = False
            if self.slot is not None:
                fs.grad_owner[self.slot] = self
            return
        op = dist.ReduceOp.AVG if (fs.use_avg and fs.ws > 1) else dist.ReduceOp.SUM  # (1 rank: sum)
        self.rs_work = dist.reduce_scatter_tensor(fs.grad_chunk(self), self.gfull, op=op, group=fs.pg,
                                                  async_op=True)
        if fs.offload and fs.copy_stream is not None and not fs.opt_on_device:
            # the averaged shard gradient goes back to pinned host memory on the copy stream as
            # soon as its reduce-scatter lands, overlapping the rest of backward
            with torch.cuda.stream(fs.copy_stream):
                self.rs_work.wait()
                lo, hi = self.shard_off, self.shard_off + self.chunk
                fs.shard_grad[lo:hi].copy_(fs.stage_grad[lo:hi], non_blocking=True)
        # at most two unit gradient buffers alive: the previously launched reduce-scatter
        # is ordered before further compute (a stream wait on RCCL) and its buffer released
        prev = fs.last_rs
        if prev is not None and prev is not self and prev.rs_work is not None:
            prev.rs_work.wait()
            prev.rs_work = None
            prev._free(prev.gfull)
        fs.last_rs = self
        for _, p in self.params:
            p.grad = None
        self.grads_live = False
        if not self.root:
            self.reshard()

    def finish(self):
        if self.grads_live:
            self.reduce()
        if self.rs_work is not None:
            self.rs_work.wait()
            self.rs_work = None
            self._free(self.gfull)
        self.bwd_started = False


class FullyShardedDP:
    sharded_optimizer = True

    def __init__(self, model: nn.Module, device=None, units=None, mode="flat", offload=False, process_group=None,
                 prefetch=True, engine_units=(), static=False, param_dtype=None, reshard_after_forward=True,
                 offload_optimizer="host"):
        """units: [(name, module)] (None: ``default_units``; ``[("", model)]``: the whole model
        as one unit, the reference's ``FSDP(model)`` without an auto-wrap policy); mode: 'flat' |
        'param' (NGD);
        engine_units: names of units whose forward/backward an engine drives explicitly
        (no module hooks installed on them); static: fixed-address buffers, HIP-graph capture
        (see the module docstring); reshard_after_forward (static mode): FULL_SHARD on a
        two-slot ring (True) or SHARD_GRAD_OP with every unit's buffers persistent (False)."""
        self.model = model
        self.static = bool(static)
        self.ring = self.static and bool(reshard_after_forward)
        self.param_dtype = param_dtype if param_dtype not in (None, torch.float32) else None
        self.pg = process_group
        self.ws = dist.get_world_size(process_group)
        self.rank = dist.get_rank(process_group)
        self.device = torch.device(device) if device is not None else next(model.parameters()).device
        self.use_avg = dist.get_backend(process_group) == "nccl"
        self.offload = offload
        if offload_optimizer not in ("host", "device"):
            raise ValueError(f"offload_optimizer {offload_optimizer!r}")
        self.opt_on_device = bool(offload and offload_optimizer == "device" and self.device.type == "cuda")
        self.prefetch = prefetch
        self.mode = mode
        # identical initial parameters on every rank (rank 0's), before sharding
        with torch.no_grad():
            for p in model.parameters():
                dist.broadcast(p.data, 0, group=self.pg)
        unit_list = list(units) if units is not None else default_units(model)
        # a parameter used by several units (tied weights, overlapping user units) would be
        # read by a later unit after its owner resharded it: such parameters go to the root
        # unit, which stays gathered
        seen = {}
        for ui, (name, mod) in enumerate(unit_list):
            for p in mod.parameters():
                seen.setdefault(id(p), set()).add(ui)
        owner = {}
        for ui, (name, mod) in enumerate(unit_list):
            for pn, p in mod.named_parameters():
                if p.requires_grad and id(p) not in owner and len(seen[id(p)]) == 1:
                    owner[id(p)] = (ui, f"{name}.{pn}" if name else pn)
        root_params = [(n, p) for n, p in model.named_parameters() if p.requires_grad and id(p) not in owner]
        self.units = []
        for ui, (name, mod) in enumerate(unit_list):
            ps = [(f"{name}.{pn}" if name else pn, p) for pn, p in mod.named_parameters() if p.requires_grad
                  and owner.get(id(p), (None,))[0] == ui]
            if ps:
                self.units.append(Unit(self, len(self.units), name, ps, mode))
        if root_params:
            self.units.append(Unit(self, len(self.units), "<root>", root_params, mode, root=True))
        self.by_name = {u.name: u for u in self.units}
        # shard storage: the units' chunks concatenated
        total = sum(u.chunk for u in self.units)
        sdev = torch.device("cpu") if offload else self.device
        self.shard_data = torch.zeros(total, device=sdev, dtype=torch.float32, pin_memory=offload and
                                      torch.cuda.is_available())
        self.shard_grad = torch.zeros_like(self.shard_data)
        if offload:
            self.shard_grad = self.shard_grad.pin_memory() if torch.cuda.is_available() else self.shard_grad
            self.stage_data = torch.empty(total, device=self.device)
            self.stage_grad = torch.empty(total, device=self.device)
            self.copy_stream = torch.cuda.Stream(self.device) if self.device.type == "cuda" else None
        else:
            self.copy_stream = None
        off = 0
        slots = []
        for u in self.units:
            u.shard_off = off
            lo = self.rank * u.chunk
            self.shard_data[off:off + u.chunk].copy_(u.full[lo:lo + u.chunk])
            for i, rel in u.owned:
                n, p = u.params[i]
                slots.append(Slot(n, p, off + rel, p.numel(), p.shape))
            off += u.chunk
        self.space = SpaceView(self.shard_data, self.shard_grad, slots, sdev)
        self.order = [u for u in self.units if not u.root]
        self.slot_owner, self.grad_owner, self.ring_bytes = [], [], 0
        if self.ring:
            # two slots, units alternating in forward order (neighbours -- the unit in use and
            # the one being prefetched -- never share a slot); a slot is sized for its largest
            # unit, so the gathered footprint is the two largest units (conv4_x + conv5_x for
            # ResNet-50), parameters and gradients alike.  The shards were taken above from the
            # private initial buffers, which are dropped here.
            nslot = 2 if len(self.order) > 1 else 1
            for k in range(nslot):
                size = max(u.numel for i, u in enumerate(self.order) if i % nslot == k)
                full = torch.zeros(size, device=self.device, dtype=torch.float32)
                f16 = torch.zeros(size, device=self.device, dtype=self.param_dtype) if self.param_dtype else None
                gfull = torch.zeros(size, device=self.device, dtype=torch.float32)
                for i, u in enumerate(self.order):
                    if i % nslot == k:
                        u.bind_ring(k, full, f16, gfull)
                self.ring_bytes += 2 * size * 4
            self.slot_owner, self.grad_owner = [None] * nslot, [None] * nslot
        self.stage16 = (torch.empty(total, device=self.device, dtype=self.param_dtype)
                        if self.param_dtype is not None else None)
        self.view = self.space  # (trainer interface shared with the sharded-optimizer DP)
        if self.opt_on_device:
            # the optimizer / clipper work on the device staging copies of the shard (same slots)
            self.view = SpaceView(self.stage_data, self.stage_grad, list(slots), self.device)
        self.peak_full_bytes = 0
        self.last_rs = None  # unit whose reduce-scatter was launched last
        self.engine_units = set(engine_units)
        self._hooks = []
        self._install_hooks()
        for u in self.units:
            u.reshard()
            u._free(u.gfull)
        self._account()
        model._fsdp_sharded = self  # checkpoint I/O gathers through summon_full_params

    def _quiesce(self):
        """Host code is about to touch the pinned shard: finish the copy stream's transfers."""
        if self.offload and self.copy_stream is not None:
            self.copy_stream.synchronize()

    # ------------------------------------------------------------ shard views
    def shard_chunk(self, u, lowp=False):
        c = self.shard_data[u.shard_off:u.shard_off + u.chunk]
        if self.offload:
            st = self.stage_data[u.shard_off:u.shard_off + u.chunk]
            st.copy_(c, non_blocking=True)
            c = st
        if lowp:
            c16 = self.stage16[u.shard_off:u.shard_off + u.chunk]
            c16.copy_(c)  # fp32 master shard -> bf16 wire copy
            return c16
        return c

    def grad_chunk(self, u):
        if self.offload:
            return self.stage_grad[u.shard_off:u.shard_off + u.chunk]
        return self.shard_grad[u.shard_off:u.shard_off + u.chunk]

    def _account(self):
        own = [u for u in self.units if u.slot is None]
        b = sum(u._bytes() for u in own if u.full.untyped_storage().size() != 0)
        b += sum(u._bytes() for u in own if u.gfull.untyped_storage().size() != 0)
        self.peak_full_bytes = max(self.peak_full_bytes, b + self.ring_bytes)

    def resident_param_bytes(self):
        own = sum(u._bytes() for u in self.units if u.slot is None and u.full.untyped_storage().size() != 0)
        return own + self.ring_bytes // 2

    # ------------------------------------------------------------ unit API (hooks / engine)
    def _next(self, u, step):
        i = self.order.index(u) if u in self.order else -1
        j = i + step
        return self.order[j] if 0 <= j < len(self.order) else None

    def _deferred(self, fn):
        """Run ``fn`` now, or -- while a HIP-graph capture is recording (static mode) -- as an
        action between two graph segments on every replay."""
        from . import graphs
        rec = graphs.active()
        if rec is not None:
            assert self.static, "graph capture of FSDP needs static=True"
            rec.cut([fn])
        else:
            fn()

    def pre_forward(self, name):
        if self.static:  # (a cut while a capture records, now otherwise)
            return self._deferred(lambda: self._pre_forward_now(name))
        self._pre_forward_now(name)

    def _pre_forward_now(self, name):
        u = self.by_name[name]
        for r in self.units:
            if r.root:
                r.gather(wait=True)
        u.gather(wait=True)
        if self.prefetch:
            nxt = self._next(u, +1)
            if nxt is not None:
                nxt.gather(wait=False)

    def post_forward(self, name, keep=False):
        u = self.by_name[name]
        if keep or (torch.is_grad_enabled() and u is self.order[-1]):
            return  # the backward starts with this unit
        u.reshard()

    def pre_backward(self, name):
        u = self.by_name[name]
        if self.ring:
            # FULL_SHARD on the ring: before the unit's backward segment, its gradient slot's
            # previous reduce-scatter must have read the slot, its parameters are gathered again
            # unless still resident from forward, and the previous unit is prefetched -- one
            # action between graph segments (engine units), or now (module-hook units); the
            # gradient slot is then zeroed in stream order (captured)
            self._deferred(lambda: self._ring_bwd_prepare(u))
            u.begin_backward(gather=False)
            return
        if self.static:
            # parameters are still gathered from this step's forward (SHARD_GRAD_OP keeps every
            # unit; while capturing, the forward's gathers are deferred actions, so the host
            # flag cannot tell); the gradient buffer is zeroed in stream order (captured)
            from . import graphs
            u.begin_backward(gather=(not u.gathered) and name not in self.engine_units
                             and graphs.active() is None)
            return
        u.begin_backward()
        if self.prefetch:
            prv = self._next(u, -1)
            if prv is not None and not prv.bwd_started:
                prv.gather(wait=False)

    def _ring_bwd_prepare(self, u):
        o = self.grad_owner[u.slot]
        if o is not None and o is not u and o.rs_work is not None:
            # (stream wait: the slot's reduce-scatter has read it).  rs_work stays set: under
            # graph replay it is the only per-step sign that o took part (finish_backward would
            # otherwise treat o as unused and re-reduce a zeroed slot)
            o.rs_work.wait()
        self.grad_owner[u.slot] = u
        u.gather(wait=True)
        if self.prefetch:
            prv = self._next(u, -1)
            if prv is not None:
                prv.gather(wait=False)

    def post_backward(self, name):
        u = self.by_name[name]
        if self.static and name in self.engine_units:
            from . import graphs
            if graphs.active() is not None:
                u.grads_live = False  # (host state of the capture; the action relaunches it)

                def act(u=u):
                    u.grads_live = True
                    u.reduce()
                # nothing in the graph waits for the reduce-scatter (on the ring, the next user
                # of the gradient slot waits for it in its own pre-backward action, issued after)
                return self._deferred(graphs.detached(act))
        u.reduce()

    # ------------------------------------------------------------ module hooks
    def _install_hooks(self):
        mods = dict(self.model.named_modules())
        for u in self.units:
            for _, p in u.params:
                self._hooks.append(p.register_post_accumulate_grad_hook(self._make_acc_hook(u)))
            if u.root or u.name in self.engine_units:
                continue
            m = mods[u.name]
            self._hooks.append(m.register_forward_pre_hook(self._make_pre(u)))
            self._hooks.append(m.register_forward_hook(self._make_post(u)))

    def _make_acc_hook(self, u):
        def hook(p):
            if u.name in self.engine_units:
                return  # the engine calls post_backward at the stage boundary
            if not u.bwd_started:
                # a gradient that arrived before the unit's output hook (root unit, or an
                # output without grad): start the unit's backward, keep what was accumulated
                if self.static and u.root and p.grad is not None and u.gfull.untyped_storage().data_ptr() == \
                        p.grad.untyped_storage().data_ptr():
                    # static mode, ROOT unit only: p.grad is still bound to the root's gradient
                    # buffer, which finish_backward zeroed at the end of the previous step, and
                    # autograd accumulated into it in place -- zeroing it now would drop this
                    # gradient.  (Other static units' bindings are dropped by finish_backward --
                    # a ring slot's buffer holds another unit's gradient, a SHARD_GRAD_OP unit's
                    # last step's -- so their early gradient arrives in a fresh tensor and takes
                    # the branch below.)
                    u.bwd_started = u.grads_live = True
                    u.pending = sum(1 for _, q in u.params if q.requires_grad)
                else:
                    g = p.grad
                    u.begin_backward()
                    if g is not None:
                        with torch.no_grad():
                            p.grad.add_(g)
            u.grad_ready()
        return hook

    def _make_pre(self, u):
        def pre(mod, args):
            self.pre_forward(u.name)
        return pre

    def _make_post(self, u):
        def post(mod, args, out):
            if torch.is_grad_enabled():
                fired = [False]

                def on_grad(g):
                    if not fired[0]:
                        fired[0] = True
                        self.pre_backward(u.name)
                    return g
                for t in (out if isinstance(out, (tuple, list)) else (out,)):
                    if isinstance(t, torch.Tensor) and t.requires_grad:
                        t.register_hook(on_grad)
            self.post_forward(u.name)
            return out
        return post

    # ------------------------------------------------------------ step boundary
    def finish_backward(self):
        """Complete every unit's gradient reduce-scatter (launch what is left, e.g. units
        whose parameters got no gradient), land the averaged shard gradients."""
        unused = []
        for u in self.units:
            if u.bwd_started or u.grads_live or u.rs_work is not None:
                u.finish()
            else:
                unused.append(u)
        for u in unused:  # contributes zeros (every rank must join the collective); after the
            u.begin_backward(gather=False)  # others, whose reduce-scatters may read a shared ring slot
            u.finish()
        if self.static:
            for u in self.units:
                if u.root:  # (its first gradient of the next step accumulates in place, see the hook)
                    u.gfull.zero_()
                elif u.name not in self.engine_units:
                    # module-hook units rebind p.grad to their buffer in begin_backward; until
                    # then a gradient must not accumulate into the (shared / stale) buffer
                    for _, q in u.params:
                        q.grad = None
        self.last_rs = None
        if self.offload and not self.opt_on_device:
            if self.copy_stream is not None:
                # the per-unit D2H copies were queued on the copy stream as each reduce-scatter
                # landed; the host optimizer reads the shard next
                self.copy_stream.synchronize()
            else:
                self.shard_grad.copy_(self.stage_grad, non_blocking=False)
        if not self.use_avg and self.ws > 1:
            self.view.grad.div_(self.ws)
        for u in self.units:
            if not u.root:
                u.reshard()

    def after_step(self):
        """Nothing to all-gather: the next forward gathers the updated shards (any copy still
        gathered -- the root unit, every unit in static mode -- is marked stale).  Device
        optimizer offload: the updated device shard is mirrored to the pinned host shard on the
        copy stream, ahead of the next gathers' H2D copies on that stream."""
        if self.opt_on_device:
            cs = self.copy_stream
            if cs is None:
                self.shard_data.copy_(self.stage_data)
            else:
                cs.wait_stream(torch.cuda.current_stream(self.device))
                with torch.cuda.stream(cs):
                    self.shard_data.copy_(self.stage_data, non_blocking=True)
        for u in self.units:
            if u.root or self.static:
                u.gathered = False
            else:
                u.reshard()

    def sync_buffers(self, src: int = 0):
        from .dist import broadcast_buffers
        broadcast_buffers(self.model, src, self.pg)

    @contextlib.contextmanager
    def summon_full_params(self):
        """All units gathered (checkpointing / state_dict) with the exact fp32 masters (also
        under a bf16 param_dtype); resharded on exit.  Not available on the full-shard ring
        (units share slots): use ``full_state_dict`` / ``load_full_state_dict``, which stream
        unit by unit."""
        if self.ring:
            raise RuntimeError("summon_full_params: full-shard ring mode holds two units at a time; "
                               "use full_state_dict() / load_full_state_dict()")
        for u in self.units:
            if u.full16 is not None:
                if u.work is not None:
                    u.gather(wait=True)  # finish an in-flight (bf16) prefetch first ...
                u.gathered = False       # ... a bf16-rounded gather is not the master copy
            u.gather(wait=True, exact=True)
        try:
            yield
        finally:
            for u in self.units:
                u.reshard()

    def load_full_state_dict(self, sd, strict=True):
        """Load a full (reference-schema) state_dict: every rank keeps its shard of it."""
        if self.ring:
            return self._ring_load(sd, strict)
        with self.summon_full_params():
            res = self.model.load_state_dict(sd, strict=strict)
            with torch.no_grad():
                for u in self.units:
                    lo = self.rank * u.chunk
                    self._quiesce()
                    self.shard_data[u.shard_off:u.shard_off + u.chunk].copy_(u.full[lo:lo + u.chunk])
        return res

    def full_state_dict(self):
        if self.ring:
            return self._ring_state_dict()
        with self.summon_full_params():
            return {k: v.detach().clone().cpu() for k, v in self.model.state_dict().items()}

    def _drop_lowp_gathers(self):
        """A unit still gathered from a bf16 wire (e.g. after an eval forward) holds rounded
        parameters, not the fp32 masters: finish any in-flight gather, then mark it stale so
        the next exact gather re-fetches the shards (as ``summon_full_params`` does)."""
        for u in self.units:
            if u.full16 is not None:
                if u.work is not None:
                    u.gather(wait=True)
                u.gathered = False

    def _ring_state_dict(self):
        """Unit by unit: exact fp32 gather into the unit's slot, copy out (collective)."""
        vals = {}
        self._drop_lowp_gathers()
        for u in self.units:
            u.gather(wait=True, exact=True)
            for _, p in u.params:
                vals[id(p)] = p.detach().clone().cpu()
        for u in self.units:  # (exact masters are not the bf16-wire values forward expects)
            if u.slot is not None:
                u.gathered = False
        return {k: (vals[id(v)] if id(v) in vals else v.detach().clone().cpu())
                for k, v in self.model.state_dict(keep_vars=True).items()}

    @torch.no_grad()
    def _ring_load(self, sd, strict):
        keys = list(self.model.state_dict(keep_vars=True).keys())
        missing = [k for k in keys if k not in sd]
        unexpected = [k for k in sd if k not in set(keys)]
        if strict and (missing or unexpected):
            raise RuntimeError(f"load_full_state_dict: missing {missing[:5]}, unexpected {unexpected[:5]}")
        self._drop_lowp_gathers()
        for u in self.units:
            # the slot must hold THIS unit's current values before the keys of ``sd`` are written
            # over it (a key missing with strict=False keeps them; claiming the slot alone
            # would leave the previous owner's parameters there)
            u.gather(wait=True, exact=True)
            for n, p in u.params:
                if n in sd:
                    p.data.copy_(sd[n].to(p.device, p.dtype).view(p.shape))
            lo = self.rank * u.chunk
            self._quiesce()
            self.shard_data[u.shard_off:u.shard_off + u.chunk].copy_(u.full[lo:lo + u.chunk])
            if u.slot is not None:
                u.gathered = False
        for n, b in self.model.named_buffers():
            if n in sd:
                b.copy_(sd[n].to(b.device, b.dtype).view(b.shape))
        return missing, unexpected

    def remove(self):
        for h in self._hooks:
            h.remove()
        self._hooks = []
