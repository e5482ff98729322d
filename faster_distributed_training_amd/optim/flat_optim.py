"""Fused optimizers over the flat parameter buffer (``utils/flat.py``).

Each optimizer is a real ``torch.optim.Optimizer`` (so ``torch.optim.lr_scheduler``
works unchanged: MultiStepLR / CosineAnnealingLR / OneCycleLR / StepLR as the
reference uses, survey A10) whose ``step`` is ONE HIP launch over the whole model:
grad * clip-coefficient (device scalar) -> found-inf skip (device flag) -> weight decay
-> update -> bf16 shadow write -> grad zeroing (``csrc/kernels/optim.hip``).
The CPU path runs the same math with torch ops (also the kernel-test oracle).

Reference update rules:
* SGD / momentum / dampening / nesterov: ``ngd_optimizer.py:478-506`` (the NGD tail) and
  ``tuning/resnet50_tuning.py:437`` (plain SGD);
* MADGRAD (``resnet50_test.py:493``) and MirrorMADGRAD (``transformer_test.py:220``) come
  from the external ``madgrad`` package, which is not installed here: MADGRAD follows
  Defazio & Jelassi 2021 (dual averaging, cube-root denominator, momentum as primal
  averaging, x0 recomputed when momentum == 0); MirrorMADGRAD uses the mirror-descent
  form z <- z - lamb*g/rms_{k+1}, p <- (1-ck) p + ck z.  Parity with the package is
  unpinned (no copy available offline); see tests/test_optim.py.
"""
from __future__ import annotations

import math

import torch

from ..ops import _native
from ..utils.flat import FlatParams


def _sp():
    return _native.stream_ptr()


def _p(t):
    return 0 if t is None else t.data_ptr()


def _layout_key(flat) -> str:
    """Fingerprint of a flat buffer's slot order (names, offsets, sizes): flat optimizer state
    is only meaningful for the layout it was saved with."""
    import hashlib
    h = hashlib.sha1()
    for sl in getattr(flat, "slots", []):
        h.update(f"{sl.name}:{sl.offset}:{sl.numel};".encode())
    return h.hexdigest()


def _slot_table(flat) -> list:
    return [(sl.name, int(sl.offset), int(sl.numel)) for sl in getattr(flat, "slots", [])]


def _slot_remap(saved, flat):
    """Function moving a saved per-element state vector (slot table ``saved``) onto ``flat``'s
    slot order, matched by slot name; refuses a table whose names / sizes do not match."""
    cur = {n: (o, k) for n, o, k in _slot_table(flat)}
    old = {n: (o, k) for n, o, k in saved}
    if set(cur) != set(old) or any(cur[n][1] != old[n][1] for n in cur):
        raise ValueError("optimizer state was saved for different parameters (slot names / sizes differ)")
    if all(cur[n][0] == old[n][0] for n in cur):
        return lambda v: v
    pairs = [(old[n][0], cur[n][0], cur[n][1]) for n in cur]

    def move(v):
        out = torch.zeros(flat.numel, dtype=v.dtype, device=v.device)
        for so, do, k in pairs:
            out[do:do + k].copy_(v[so:so + k])
        return out
    return move


class FlatOptimizer(torch.optim.Optimizer):
    def __init__(self, flat: FlatParams, defaults: dict, zero_grad_in_step: bool = True):
        self.flat = flat
        # the update runs over the flat buffer; torch.optim.Optimizer only needs a parameter
        # list for its param_groups bookkeeping (a flat FSDP shard may hold no whole one)
        super().__init__(flat.params or [torch.nn.Parameter(torch.zeros(0))], defaults)
        self.zero_grad_in_step = zero_grad_in_step
        self.k = 0  # step() calls
        # steps skipped on the device (non-finite / fp16 overflow): the kernels bump it and
        # use k - kskip as their step count, like torch's GradScaler which never calls
        # optimizer.step() on a skipped step (so MADGRAD's lamb / Adam's bias correction
        # only advance on applied steps) -- no host sync
        self.kskip = torch.zeros(1, device=flat.device, dtype=torch.int32)
        self._native = flat.data.is_cuda and _native.enabled()

    @property
    def group(self):
        return self.param_groups[0]

    def zero_grad(self, set_to_none: bool = False):  # noqa: ARG002 - views must persist
        self.flat.zero_grad()

    def _state_buf(self, name, init="zeros"):
        st = self.state.setdefault("__flat__", {})
        if name not in st:
            if init == "zeros":
                st[name] = torch.zeros_like(self.flat.data)
            elif init == "copy":
                st[name] = self.flat.data.clone()
        return st[name]

    def step(self, closure=None, grad_scale: torch.Tensor | None = None, found_inf: torch.Tensor | None = None):
        loss = closure() if closure is not None else None
        self._packed = False
        self._step(grad_scale, found_inf)
        plan = self._pack_plan()
        if plan is not None:  # the packed conv layouts follow the weights only after a fused step
            if self._packed:
                plan.mark_opt_packed(self.flat)
            else:
                plan.invalidate_pack()
        self.k += 1
        return loss

    # ------------------------------------------------------------ fused conv weight repack
    # When the flat buffer holds the weights of a native-engine ResNet (``flat.pack_owner``, set
    # by the trainer), SGD / MADGRAD steps also write the convolutions' packed bf16 layouts
    # (csrc/kernels/optim_pack.hip) and the next forward skips its repack pass.
    def _pack_plan(self):
        return getattr(getattr(self.flat, "pack_owner", None), "_plan", None)

    def _pack_args(self):
        """Trailing table arguments of each fused update-and-pack launch (a list), or None."""
        plan = self._pack_plan()
        if plan is None or not self._native:
            return None
        return plan.update_table(self.flat)

    # ------------------------------------------------------------ state dict
    # The optimizer state lives in whole-model flat buffers (self.state["__flat__"]), which
    # torch.optim.Optimizer.state_dict() would not serialise (its state is keyed by
    # parameter); save and restore them explicitly.
    def state_dict(self):
        groups = [{k: v for k, v in g.items() if k != "params"} for g in self.param_groups]
        flat = {k: (v.detach().clone() if torch.is_tensor(v) else v)
                for k, v in self.state.get("__flat__", {}).items()}
        return {"flat_state": flat, "param_groups": groups, "k": self.k, "kskip": self.kskip.detach().clone().cpu(),
                "numel": self.flat.numel, "layout": _layout_key(self.flat), "slots": _slot_table(self.flat)}

    def load_state_dict(self, sd):
        if "flat_state" not in sd:  # a plain torch.optim state dict: hyper-parameters only
            for g, sg in zip(self.param_groups, sd.get("param_groups", [])):
                g.update({k: v for k, v in sg.items() if k != "params"})
            return
        remap = None
        if "slots" in sd:
            # per-slot (name, offset, numel): the saved vectors are moved slot by slot onto THIS
            # buffer's order (a checkpoint from before a slot reordering, e.g. the transformer's
            # flat_adjacent groups, lands on the right parameters)
            remap = _slot_remap(sd["slots"], self.flat)
        elif "layout" in sd:
            if sd["layout"] != _layout_key(self.flat):
                # same element count, other slot order: the flat state vectors would be applied
                # to the wrong parameters
                raise ValueError("optimizer state was saved for a different parameter order")
        else:
            # no slot table and no fingerprint (written before either existed): the numel check
            # cannot tell a reordered buffer from the same one (every slot is padded on its own)
            raise ValueError("flat optimizer state carries no slot table or layout fingerprint: its parameter "
                             "order cannot be verified (re-save it, or load the model weights only)")
        if sd.get("numel", self.flat.numel) != self.flat.numel and remap is None:
            raise ValueError("optimizer state was saved for a different parameter layout")
        for g, sg in zip(self.param_groups, sd["param_groups"]):
            g.update(sg)
        st = self.state.setdefault("__flat__", {})
        for k, v in sd["flat_state"].items():
            if torch.is_tensor(v) and remap is not None and v.dim() == 1 and v.numel() == sd.get("numel", -1):
                v = remap(v)
            st[k] = v.to(self.flat.device) if torch.is_tensor(v) else v
        self.k = int(sd.get("k", 0))
        if "kskip" in sd:
            self.kskip.copy_(sd["kskip"].to(self.kskip.device))

    @property
    def applied_k(self) -> int:
        """Applied steps so far (host view; syncs -- CPU path / tests only)."""
        return self.k - int(self.kskip.item())

    def _cpu_common(self, grad_scale, found_inf):
        if found_inf is not None and bool(found_inf.item() != 0):
            self.kskip += 1
            if self.zero_grad_in_step:  # a skipped step still clears the gradient
                self.flat.grad.zero_()
            return None
        g = self.flat.grad
        if grad_scale is not None:
            g = g * grad_scale.to(g.device)
        return g

    def _finish_cpu(self):
        self.flat.refresh_shadow()
        if self.zero_grad_in_step:
            self.flat.grad.zero_()


class SGD(FlatOptimizer):
    def __init__(self, flat, lr=0.1, momentum=0.0, dampening=0.0, weight_decay=0.0, nesterov=False, **kw):
        if nesterov and (momentum <= 0 or dampening != 0):
            raise ValueError("Nesterov momentum requires a momentum and zero dampening")
        super().__init__(flat, dict(lr=lr, momentum=momentum, dampening=dampening, weight_decay=weight_decay,
                                    nesterov=nesterov), **kw)

    def _step(self, grad_scale, found_inf, d_override=None):
        g = self.group
        buf = self._state_buf("momentum_buffer") if g["momentum"] != 0 else None
        first = int(self.state["__flat__"].get("initialized", 0) == 0) if buf is not None else 0
        if self._native and d_override is None:
            args = [self.flat.data.data_ptr(), self.flat.grad.data_ptr(), _p(buf), _p(self.flat.shadow),
                    self.flat.numel, float(g["lr"]), float(g["momentum"]), float(g["dampening"]),
                    float(g["weight_decay"]), int(g["nesterov"]), first, _p(grad_scale), _p(found_inf),
                    int(self.zero_grad_in_step), _p(getattr(self, "lr_dev", None))]
            pk = self._pack_args()
            if pk is not None:
                for launch in pk:
                    _native.native().sgd_pack_step(*args, *launch, _sp())
                self._packed = True
            else:
                _native.native().sgd_step(*args, _sp())
        else:
            gr = self._cpu_common(grad_scale, found_inf) if d_override is None else d_override
            if gr is None:
                return
            p = self.flat.data
            d = gr + g["weight_decay"] * p if g["weight_decay"] != 0 else gr.clone()
            if buf is not None:
                if first:
                    buf.copy_(d)
                else:
                    buf.mul_(g["momentum"]).add_(d, alpha=1 - g["dampening"])
                d = d + g["momentum"] * buf if g["nesterov"] else buf
            p.add_(d, alpha=-g["lr"])
            self._finish_cpu()
        if buf is not None:
            self.state["__flat__"]["initialized"] = 1


class MADGRAD(FlatOptimizer):
    def __init__(self, flat, lr=1e-2, momentum=0.9, weight_decay=0.0, eps=1e-6, decouple_decay=False, **kw):
        if not 0.0 <= momentum < 1.0:
            raise ValueError("momentum must be in [0, 1)")
        super().__init__(flat, dict(lr=lr, momentum=momentum, weight_decay=weight_decay, eps=eps,
                                    decouple_decay=decouple_decay), **kw)

    def _step(self, grad_scale, found_inf):
        g = self.group
        gss = self._state_buf("grad_sum_sq")
        s = self._state_buf("s")
        x0 = self._state_buf("x0", init="copy") if g["momentum"] != 0 else None
        if self._native:
            args = [self.flat.data.data_ptr(), self.flat.grad.data_ptr(), gss.data_ptr(), s.data_ptr(), _p(x0),
                    _p(self.flat.shadow), self.flat.numel, float(g["lr"]), float(g["momentum"]),
                    float(g["weight_decay"]), float(g["eps"]), int(g["decouple_decay"]), self.k,
                    self.kskip.data_ptr(), _p(grad_scale), _p(found_inf), int(self.zero_grad_in_step)]
            pk = self._pack_args()
            if pk is not None:
                for launch in pk:
                    _native.native().madgrad_pack_step(*args, *launch, _sp())
                self._packed = True
            else:
                _native.native().madgrad_step(*args, _sp())
            return
        gr = self._cpu_common(grad_scale, found_inf)
        if gr is None:
            return
        p = self.flat.data
        eps, lr = g["eps"], g["lr"] + g["eps"]
        lamb = lr * math.sqrt(self.applied_k + 1)
        ck = 1 - g["momentum"]
        if g["weight_decay"] != 0 and not g["decouple_decay"]:
            gr = gr + g["weight_decay"] * p
        if g["momentum"] == 0:
            x0v = p + s / (gss.pow(1 / 3) + eps)
        else:
            x0v = x0
        gss.addcmul_(gr, gr, value=lamb)
        rms = gss.pow(1 / 3).add_(eps)
        if g["weight_decay"] != 0 and g["decouple_decay"]:
            p.mul_(1 - lr * g["weight_decay"])
        s.add_(gr, alpha=lamb)
        z = x0v - s / rms
        if g["momentum"] == 0:
            p.copy_(z)
        else:
            p.mul_(1 - ck).add_(z, alpha=ck)
        self._finish_cpu()


class MirrorMADGRAD(FlatOptimizer):
    def __init__(self, flat, lr=1e-2, momentum=0.9, weight_decay=0.0, eps=0.0, decouple_decay=False, **kw):
        super().__init__(flat, dict(lr=lr, momentum=momentum, weight_decay=weight_decay, eps=eps,
                                    decouple_decay=decouple_decay), **kw)

    def _step(self, grad_scale, found_inf):
        g = self.group
        gss = self._state_buf("grad_sum_sq")
        z = self._state_buf("z", init="copy")
        if self._native:
            _native.native().mirror_madgrad_step(
                self.flat.data.data_ptr(), self.flat.grad.data_ptr(), gss.data_ptr(), z.data_ptr(),
                _p(self.flat.shadow), self.flat.numel, float(g["lr"]), float(g["momentum"]), float(g["weight_decay"]),
                float(g["eps"]), int(g["decouple_decay"]), self.k, self.kskip.data_ptr(), _p(grad_scale),
                _p(found_inf), int(self.zero_grad_in_step), _sp())
            return
        gr = self._cpu_common(grad_scale, found_inf)
        if gr is None:
            return
        p = self.flat.data
        eps, lr = g["eps"], g["lr"] + g["eps"]
        lamb = lr * math.sqrt(self.applied_k + 1)
        ck = 1 - g["momentum"]
        if g["weight_decay"] != 0 and not g["decouple_decay"]:
            gr = gr + g["weight_decay"] * p
        gss.addcmul_(gr, gr, value=lamb)
        rms = gss.pow(1 / 3).add_(eps)
        step = torch.where(rms > 0, lamb * gr / torch.where(rms > 0, rms, torch.ones_like(rms)), torch.zeros_like(rms))
        z.sub_(step)
        if g["weight_decay"] != 0 and g["decouple_decay"]:
            z.mul_(1 - lr * g["weight_decay"])
        p.mul_(1 - ck).add_(z, alpha=ck)
        self._finish_cpu()


class Adam(FlatOptimizer):
    def __init__(self, flat, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0, adamw=False, **kw):
        super().__init__(flat, dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay, adamw=adamw), **kw)

    def _step(self, grad_scale, found_inf):
        g = self.group
        m = self._state_buf("exp_avg")
        v = self._state_buf("exp_avg_sq")
        b1, b2 = g["betas"]
        if self._native:
            _native.native().adam_step(
                self.flat.data.data_ptr(), self.flat.grad.data_ptr(), m.data_ptr(), v.data_ptr(), _p(self.flat.shadow),
                self.flat.numel, float(g["lr"]), float(b1), float(b2), float(g["eps"]), float(g["weight_decay"]),
                int(g["adamw"]), self.k + 1, self.kskip.data_ptr(), _p(grad_scale), _p(found_inf),
                int(self.zero_grad_in_step), _sp())
            return
        gr = self._cpu_common(grad_scale, found_inf)
        if gr is None:
            return
        step = self.applied_k + 1
        p = self.flat.data
        if g["weight_decay"] != 0:
            if g["adamw"]:
                p.mul_(1 - g["lr"] * g["weight_decay"])
            else:
                gr = gr + g["weight_decay"] * p
        m.mul_(b1).add_(gr, alpha=1 - b1)
        v.mul_(b2).addcmul_(gr, gr, value=1 - b2)
        p.addcdiv_(m / (1 - b1 ** step), (v / (1 - b2 ** step)).sqrt_().add_(g["eps"]), value=-g["lr"])
        self._finish_cpu()


# ------------------------------------------------------------------ clipping / AMP
class GradClipper:
    """clip_grad_norm_ over the flat gradient with the result kept ON DEVICE
    (``coef`` is passed to the optimizer kernel): no host sync, unlike
    ``torch.nn.utils.clip_grad_norm_`` + GradScaler's found_inf check in the reference
    (``resnet50_test.py:544-548``).  Also performs GradScaler's unscale + inf check."""

    def __init__(self, flat: FlatParams, nblocks: int = 1024, process_group=None, sharded: bool = False):
        self.flat = flat
        self.sharded = sharded  # FSDP: grads are a per-rank shard -> all-reduce the sum of squares
        self.pg = process_group
        dev = flat.device
        self.nb = nblocks
        self.part = torch.empty(nblocks, device=dev, dtype=torch.float32)
        self.out = torch.zeros(2, device=dev, dtype=torch.float32)  # [norm, coef]
        self.found_inf = torch.zeros(1, device=dev, dtype=torch.int32)
        self.total = torch.zeros(1, device=dev, dtype=torch.float64)  # sharded: fp64 sum of squares

    @property
    def norm(self):
        return self.out[0]

    @property
    def coef(self):
        return self.out[1:2]

    def __call__(self, max_norm: float, inv_scale: torch.Tensor | None = None, check_inf: bool = False):
        g = self.flat.grad
        if g.is_cuda and _native.enabled():
            nat = _native.native()
            if check_inf:
                self.found_inf.zero_()
            nat.grad_sumsq(g.data_ptr(), g.numel(), _p(inv_scale), int(inv_scale is not None), self.part.data_ptr(),
                           self.nb, _p(self.found_inf) if check_inf else 0, _sp())
            if self.sharded:
                # fp64 total with the unsharded finalize's summation tree, all-reduced in fp64:
                # one rank reproduces the unsharded norm / coefficient bitwise
                nat.grad_norm_finalize(self.part.data_ptr(), self.nb, float(max_norm), self.out.data_ptr(),
                                       self.total.data_ptr(), 1, _sp())
                import torch.distributed as dist
                dist.all_reduce(self.total, group=self.pg)
                nat.grad_norm_finalize(self.part.data_ptr(), self.nb, float(max_norm), self.out.data_ptr(),
                                       self.total.data_ptr(), 2, _sp())
                return self.out[0]
            nat.grad_norm_finalize(self.part.data_ptr(), self.nb, float(max_norm), self.out.data_ptr(), 0, 0, _sp())
        else:
            if inv_scale is not None:
                g.mul_(inv_scale)
            if check_inf:
                self.found_inf.fill_(int(not torch.isfinite(g).all()))
            if self.sharded:
                return self._sharded_finalize(g.double().pow(2).sum().float(), max_norm)
            norm = g.double().pow(2).sum().sqrt()
            self.out[0] = norm.float()
            c = (max_norm / (norm + 1e-6)).clamp(max=1.0) if max_norm > 0 else torch.ones((), dtype=torch.float64)
            self.out[1] = c.float()
        return self.out[0]

    def _sharded_finalize(self, sumsq, max_norm):
        import torch.distributed as dist
        t = sumsq.reshape(1).float()
        if not t.is_cuda and dist.get_backend(self.pg) == "nccl":  # host-offloaded shard on RCCL
            t = t.cuda()
        dist.all_reduce(t, group=self.pg)
        t = t.to(self.out.device)
        norm = t.sqrt()
        coef = (max_norm / (norm + 1e-6)).clamp(max=1.0) if max_norm > 0 else torch.ones_like(norm)
        self.out[0:1].copy_(norm)
        self.out[1:2].copy_(coef)
        return self.out[0]


class DeviceGradScaler:
    """fp16 loss scaling with all state on the device (replaces
    ``torch.cuda.amp.GradScaler`` / fairscale ``ShardedGradScaler``,
    ``resnet50_test.py:705-706``, ``transformer_test.py:368``).  ``found_inf`` is
    all-reduced (MAX) across ranks when distributed, like ShardedGradScaler."""

    def __init__(self, device, init_scale=2.0**16, growth_factor=2.0, backoff_factor=0.5, growth_interval=2000,
                 enabled=True):
        self.enabled = enabled
        self.scale = torch.full((1,), init_scale if enabled else 1.0, device=device, dtype=torch.float32)
        self.growth_tracker = torch.zeros(1, device=device, dtype=torch.int32)
        self.gf, self.bf, self.gi = growth_factor, backoff_factor, growth_interval

    def scale_loss(self, loss):
        return loss * self.scale.to(loss.dtype) if self.enabled else loss

    def inv_scale(self):
        return (1.0 / self.scale) if self.enabled else None

    def sync_found_inf(self, found_inf):
        import torch.distributed as dist
        if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
            dist.all_reduce(found_inf, op=dist.ReduceOp.MAX)

    def update(self, found_inf):
        if not self.enabled:
            return
        torch._amp_update_scale_(self.scale, self.growth_tracker, found_inf.float(), self.gf, self.bf, self.gi)

    def state_dict(self):
        return {"scale": self.scale.clone(), "growth_tracker": self.growth_tracker.clone()}

    def load_state_dict(self, sd):
        self.scale.copy_(sd["scale"])
        self.growth_tracker.copy_(sd["growth_tracker"])
