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
        if ctx.needs_input_grad[1]:
            dw = wgrad(g2, x2).to(wd)
        if bd is not None and ctx.needs_input_grad[2]:
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
