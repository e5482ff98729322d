"""Linear layer with an MI355X-shaped weight gradient (transformer projections / FFN).

Under autograd the weight gradient of ``y = x W^T + b`` is ``dW = dY^T X``: an (out x in)
output -- 512 x 512 ... 1536 x 512 here -- reduced over all B*L tokens (32K at bs 256,
L 128).  The library GEMM PyTorch issues for it tiles the small output into 50-70 workgroups
that each walk the whole 32K-deep reduction: ~200 us per call on MI355X, 0.2-0.3 PFLOP/s,
24 calls per transformer step (measured, ``scripts/bench_linear_wgrad.py``).

Here the reduction is split over the batch dimension of a strided-batched GEMM (S slices of
the token axis, each an (out x in) product over M/S tokens, hundreds of workgroups), the
slices written in fp32 (``out_dtype``) and summed: 35-76 us per call, and dW comes out in
fp32 straight for the fp32 master gradient (no bf16 rounding of the gradient, no cast).
Forward and the data gradient stay single library GEMMs (their M = tokens is large).

Reference: the projections are plain ``nn.Linear`` (``transformer.py:159-227``); parameters
and state-dict names are unchanged -- only the autograd formula is replaced.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F


def _splits(M: int) -> int:
    for s in (16, 8, 4, 2):
        if M % s == 0 and M // s >= 1024:
            return s
    return 1


def wgrad(gy: torch.Tensor, x: torch.Tensor) -> torch.Tensor:
    """dW = gy^T x in fp32 for gy [M, out], x [M, in] (bf16 on the GPU)."""
    M = gy.shape[0]
    s = _splits(M)
    try:
        if s == 1:
            return torch.mm(gy.t(), x, out_dtype=torch.float32)
        p = torch.bmm(gy.view(s, M // s, -1).transpose(1, 2), x.view(s, M // s, -1), out_dtype=torch.float32)
        return p.sum(0)
    except (TypeError, RuntimeError):  # no out_dtype support: bf16 slices, fp32 sum
        if s == 1:
            return (gy.t() @ x).float()
        return torch.bmm(gy.view(s, M // s, -1).transpose(1, 2), x.view(s, M // s, -1)).float().sum(0)


# ------------------------------------------------------------------ direct gradients
# With flat gradient storage (utils/flat.py) every parameter's ``.grad`` is a static fp32
# view that autograd accumulates into with one extra add kernel per parameter (~120 per
# transformer step, 0.9 ms measured).  Parameters flagged by ``enable_direct_grads`` get
# their weight / bias / LayerNorm gradients folded straight into that view by the kernel
# that finishes the reduction; the backward then returns None for them and fires the
# grad-ready hooks itself (DDP bucket readiness, ops/resnet_fused.py grad_ready).
def enable_direct_grads(params, on: bool = True) -> None:
    for p in params:
        p._fdt_direct = on


def direct_target(p):
    """The fp32 gradient view to accumulate into, or None (autograd returns the gradient)."""
    if p is None or not getattr(p, "_fdt_direct", False) or not p.is_leaf:
        return None
    g = p.grad
    if g is None or g.dtype != torch.float32 or not g.is_contiguous() or not g.is_cuda:
        return None
    return g


def enable_shadow_weights(flat) -> None:
    """Point every parameter at its bf16 shadow in ``flat`` (utils/flat.py: rewritten by the
    optimizer kernel each step), so bf16 compute reads it instead of casting the fp32 master
    weight each forward (~50 cast kernels per transformer step)."""
    if flat.shadow is None:
        return
    for s in flat.slots:
        s.param._fdt_shadow = flat.shadow_view(s.param)


def cast_weight(w: torch.Tensor, dt) -> torch.Tensor:
    sh = getattr(w, "_fdt_shadow", None)
    if sh is not None and dt == torch.bfloat16 and w.dtype == torch.float32:
        return sh
    return w.to(dt)


def _native_ok(t) -> bool:
    from . import _native
    return _native.use_native(t) and hasattr(_native.native(), "slab_sum_acc")


def slab_sum_into(src: torch.Tensor, dst: torch.Tensor) -> None:
    """dst += src.sum(0) for fp32 src [s, *dst.shape] (one HIP pass)."""
    from . import _native
    src = src.contiguous()
    n = dst.numel()
    if _native_ok(dst) and n % 4 == 0:
        _native.native().slab_sum_acc(src.data_ptr(), dst.data_ptr(), src.shape[0], n, n, _native.stream_ptr())
    else:
        dst.add_(src.view(src.shape[0], *dst.shape).sum(0))


def mark_ready(p) -> None:
    from .resnet_fused import grad_ready
    grad_ready(p)


def wgrad_into(gy: torch.Tensor, x: torch.Tensor, dst: torch.Tensor) -> None:
    """dst += gy^T x (fp32 dst): split-K slabs folded into dst by one kernel."""
    M = gy.shape[0]
    s = _splits(M)
    if s > 1 and _native_ok(dst):
        try:
            p = torch.bmm(gy.view(s, M // s, -1).transpose(1, 2), x.view(s, M // s, -1), out_dtype=torch.float32)
            slab_sum_into(p, dst)
            return
        except (TypeError, RuntimeError):
            pass
    dst.add_(wgrad(gy, x).view_as(dst))


def bias_grad_into(gy: torch.Tensor, dst: torch.Tensor) -> None:
    """dst += column sums of gy [M, out] (the colsum kernel accumulates atomically)."""
    from . import _native
    if (gy.dtype == torch.bfloat16 and gy.stride(1) == 1 and gy.stride(0) % 8 == 0 and gy.data_ptr() % 16 == 0
            and gy.shape[1] % 8 == 0 and _native.use_native(gy) and hasattr(_native.native(), "colsum_bf16")
            and dst.numel() == gy.shape[1]):
        _native.native().colsum_bf16(gy.data_ptr(), dst.data_ptr(), gy.shape[0], gy.shape[1], gy.stride(0),
                                     _native.stream_ptr())
    else:
        dst.add_(gy.sum(0, dtype=torch.float32).view_as(dst))


def bias_grad(gy: torch.Tensor) -> torch.Tensor:
    """db = sum over tokens of gy [M, out] in fp32: one streaming HIP pass (csrc/kernels/
    mlp.hip colsum_bf16; PyTorch's column reduction runs at ~1/3 of HBM bandwidth here, a
    GEMV against a ones vector with fp32 output takes ~11 ms -- both measured)."""
    from . import _native
    if (gy.dtype == torch.bfloat16 and gy.is_contiguous() and gy.shape[1] % 8 == 0 and _native.use_native(gy)
            and hasattr(_native.native(), "colsum_bf16")):
        out = torch.zeros(gy.shape[1], device=gy.device, dtype=torch.float32)
        _native.native().colsum_bf16(gy.data_ptr(), out.data_ptr(), gy.shape[0], gy.shape[1], 0, _native.stream_ptr())
        return out
    return gy.sum(0, dtype=torch.float32)


class _Linear(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, dt, bias_grad=True):
        xin_dtype = x.dtype
        xc = x.to(dt)
        wc = cast_weight(w, dt)
        y = F.linear(xc, wc, None if b is None else cast_weight(b, dt))
        ctx.save_for_backward(xc, wc)
        ctx.meta = (xin_dtype, w.dtype, None if b is None else b.dtype)
        ctx.params = (w, b)  # leaves whose gradient may be written in place (direct_target)
        ctx.bias_grad = bias_grad
        return y

    @staticmethod
    def backward(ctx, gy):
        xc, wc = ctx.saved_tensors
        xd, wd, bd = ctx.meta
        g2 = gy.reshape(-1, gy.shape[-1]).to(wc.dtype)
        x2 = xc.reshape(-1, xc.shape[-1])
        dx = dw = db = None
        if ctx.needs_input_grad[0]:
            dx = (g2 @ wc).view(xc.shape).to(xd)
        w, b = ctx.params
        if ctx.needs_input_grad[1]:
            tgt = direct_target(w)
            if tgt is not None:
                wgrad_into(g2, x2, tgt)
                mark_ready(w)
            else:
                dw = wgrad(g2, x2).to(wd)
        if bd is not None and ctx.needs_input_grad[2] and ctx.bias_grad:
            tgt = direct_target(b)
            if tgt is not None:
                bias_grad_into(g2, tgt)
                mark_ready(b)
            else:
                db = bias_grad(g2).to(bd)
        return dx, dw, db, None, None


def linear(x: torch.Tensor, weight: torch.Tensor, bias: torch.Tensor | None = None,
           bias_grad: bool = True) -> torch.Tensor:
    """``F.linear`` semantics (incl. autocast's compute dtype) with the split-K weight
    gradient on the GPU; plain ``F.linear`` elsewhere (CPU, fp32 compute).
    ``bias_grad=False``: the bias is added but its gradient is left to the consumer of the
    output (ops/dropout.py ``bias=``: the column sums fused into the dropout backward)."""
    b_fwd = bias if (bias_grad or bias is None) else bias.detach()
    if not x.is_cuda:
        return F.linear(x, weight, b_fwd)
    dt = torch.get_autocast_dtype("cuda") if torch.is_autocast_enabled("cuda") else x.dtype
    if dt not in (torch.bfloat16, torch.float16) or x.numel() // x.shape[-1] < 4096:
        return F.linear(x, weight, b_fwd)
    with torch.autocast("cuda", enabled=False):
        return _Linear.apply(x, weight, bias, dt, bias_grad)


def stacked(ts):
    """``torch.cat(ts, 0)`` -- as a zero-copy view when the tensors already sit back to back in
    one buffer (utils/flat.py keeps the Q / K / V shadows adjacent: ``flat_adjacent``)."""
    t0 = ts[0]
    if all(t.is_contiguous() and t.dtype == t0.dtype and t.shape[1:] == t0.shape[1:] for t in ts):
        es = t0.element_size()
        if all(ts[i + 1].data_ptr() == ts[i].data_ptr() + ts[i].numel() * es for i in range(len(ts) - 1)) and \
                all(t.untyped_storage().data_ptr() == t0.untyped_storage().data_ptr() for t in ts):
            rows = sum(t.shape[0] for t in ts)
            shape = (rows,) + tuple(t0.shape[1:])
            return t0.as_strided(shape, torch.empty(shape, device="meta").stride(), t0.storage_offset())
    return torch.cat(ts, 0)


class _LinearCat(torch.autograd.Function):
    """``F.linear(x, cat(ws), cat(bs))`` for row-stacked weights (the fused Q/K/V projection of
    three ``nn.Linear``s): the weight gradient is one split-K product over the stacked rows
    whose slabs are folded straight into each parameter's flat gradient (row-offset source,
    slab stride = the stacked size), bias gradients by row-strided column sums -- no cat
    backward split and no per-parameter accumulate kernels."""

    @staticmethod
    def forward(ctx, x, dt, n, *params):
        ws, bs = params[:n], params[n:]
        xc = x.to(dt)
        wc = stacked([cast_weight(w, dt) for w in ws])
        bc = stacked([cast_weight(b, dt) for b in bs]) if bs else None
        y = F.linear(xc, wc, bc)
        ctx.save_for_backward(xc, wc)
        ctx.params = (ws, bs)
        ctx.xd = x.dtype
        return y

    @staticmethod
    def backward(ctx, gy):
        from . import _native
        xc, wc = ctx.saved_tensors
        ws, bs = ctx.params
        n = len(ws)
        g2 = gy.reshape(-1, gy.shape[-1]).to(wc.dtype)
        x2 = xc.reshape(-1, xc.shape[-1])
        dx = (g2 @ wc).view(xc.shape).to(ctx.xd) if ctx.needs_input_grad[0] else None
        rows = [w.shape[0] for w in ws]
        offs = [sum(rows[:i]) for i in range(n)]
        gw = [None] * n
        if any(ctx.needs_input_grad[3:3 + n]):
            tg = [direct_target(w) for w in ws]
            M, K, R = g2.shape[0], x2.shape[1], wc.shape[0]
            s = _splits(M)
            done = False
            if all(t is not None for t in tg) and s > 1 and _native_ok(g2) and K % 4 == 0:
                try:
                    p = torch.bmm(g2.view(s, M // s, -1).transpose(1, 2), x2.view(s, M // s, -1),
                                  out_dtype=torch.float32)
                    if all(tg[i + 1].data_ptr() == tg[i].data_ptr() + rows[i] * K * 4 for i in range(n - 1)):
                        # the parameters' gradients are adjacent (utils/flat.py flat_adjacent): one pass
                        _native.native().slab_sum_acc(p.data_ptr(), tg[0].data_ptr(), s, R * K, R * K,
                                                      _native.stream_ptr())
                    else:
                        for i in range(n):
                            _native.native().slab_sum_acc(p.data_ptr() + offs[i] * K * 4, tg[i].data_ptr(), s,
                                                          R * K, rows[i] * K, _native.stream_ptr())
                    done = True
                except (TypeError, RuntimeError):
                    done = False
            if done:
                for w in ws:
                    mark_ready(w)
            else:
                dw = wgrad(g2, x2)
                for i, w in enumerate(ws):
                    part = dw[offs[i]:offs[i] + rows[i]]
                    if tg[i] is not None:
                        tg[i].add_(part)
                        mark_ready(w)
                    else:
                        gw[i] = part.to(w.dtype)
        gb = [None] * len(bs)
        for i, b in enumerate(bs):
            if not ctx.needs_input_grad[3 + n + i]:
                continue
            cols = g2[:, offs[i]:offs[i] + rows[i]]
            tgt = direct_target(b)
            if tgt is not None:
                bias_grad_into(cols, tgt)
                mark_ready(b)
            else:
                gb[i] = bias_grad(cols.contiguous()).to(b.dtype)
        return (dx, None, None, *gw, *gb)


def linear_cat(x: torch.Tensor, weights, biases=None) -> torch.Tensor:
    """``F.linear(x, cat(weights), cat(biases))`` with per-parameter gradients (see _LinearCat)."""
    biases = list(biases) if biases is not None else []
    if x.is_cuda:
        dt = torch.get_autocast_dtype("cuda") if torch.is_autocast_enabled("cuda") else x.dtype
        if dt in (torch.bfloat16, torch.float16) and x.numel() // x.shape[-1] >= 4096:
            with torch.autocast("cuda", enabled=False):
                return _LinearCat.apply(x, dt, len(weights), *weights, *biases)
    return F.linear(x, torch.cat(list(weights), 0), torch.cat(biases, 0) if biases else None)
