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
    if (gy.dtype == torch.bfloat16 and gy.is_contiguous() and gy.shape[1] % 8 == 0 and _native.use_native(gy)
            and hasattr(_native.native(), "colsum_bf16") and dst.numel() == gy.shape[1]):
        _native.native().colsum_bf16(gy.data_ptr(), dst.data_ptr(), gy.shape[0], gy.shape[1], _native.stream_ptr())
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
        _native.native().colsum_bf16(gy.data_ptr(), out.data_ptr(), gy.shape[0], gy.shape[1], _native.stream_ptr())
        return out
    return gy.sum(0, dtype=torch.float32)


class _Linear(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, dt):
        xin_dtype = x.dtype
        xc = x.to(dt)
        wc = w.to(dt)
        y = F.linear(xc, wc, None if b is None else b.to(dt))
        ctx.save_for_backward(xc, wc)
        ctx.meta = (xin_dtype, w.dtype, None if b is None else b.dtype)
        ctx.params = (w, b)  # leaves whose gradient may be written in place (direct_target)
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
        if bd is not None and ctx.needs_input_grad[2]:
            tgt = direct_target(b)
            if tgt is not None:
                bias_grad_into(g2, tgt)
                mark_ready(b)
            else:
                db = bias_grad(g2).to(bd)
        return dx, dw, db, None


def linear(x: torch.Tensor, weight: torch.Tensor, bias: torch.Tensor | None = None) -> torch.Tensor:
    """``F.linear`` semantics (incl. autocast's compute dtype) with the split-K weight
    gradient on the GPU; plain ``F.linear`` elsewhere (CPU, fp32 compute)."""
    if not x.is_cuda:
        return F.linear(x, weight, bias)
    dt = torch.get_autocast_dtype("cuda") if torch.is_autocast_enabled("cuda") else x.dtype
    if dt not in (torch.bfloat16, torch.float16) or x.numel() // x.shape[-1] < 4096:
        return F.linear(x, weight, bias)
    with torch.autocast("cuda", enabled=False):
        return _Linear.apply(x, weight, bias, dt)
