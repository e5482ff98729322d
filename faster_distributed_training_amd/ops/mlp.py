"""FusedMLP: Linear -> ReLU -> Linear as one autograd op (reference ``MLPScratch``,
``transformer.py:292-338``).

The reference backward runs a per-element Python loop with a host sync per element
(survey Q6) and averages the bias gradients over the batch (Q5).  Here the ReLU mask,
bias add and bias-gradient reduction are fused: forward is ``GEMM -> (bias+ReLU) ->
GEMM(+bias)``; backward is ``GEMM -> (mask + column-sum) -> GEMM x2``.  On GPU the
elementwise+reduction steps are one HIP kernel each (``csrc/kernels/mlp.hip``);
``bias_grad_mean=True`` reproduces the reference's 1/B bias gradients.
"""
from __future__ import annotations

import torch

from . import _native


def _flat2(x):
    return x.reshape(-1, x.shape[-1])


class FusedMLPFunction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, X, W1, b1, W2, b2, bias_grad_mean):
        dt = torch.get_autocast_dtype(X.device.type) if torch.is_autocast_enabled(X.device.type) else X.dtype
        x2 = _flat2(X).to(dt)
        w1, w2 = W1.to(dt), W2.to(dt)
        pre = x2 @ w1.t()
        nat = _native.load() if _native.use_native(X) else None
        if nat is not None and hasattr(nat, "bias_relu_fwd") and pre.is_contiguous():
            # one pass: pre += b1 (in place, kept for the ReLU mask); act = relu(pre)
            act = torch.empty_like(pre)
            b1f = b1.float().contiguous() if b1 is not None else None
            nat.bias_relu_fwd(pre.data_ptr(), _native.ptr(b1f), act.data_ptr(),
                              pre.shape[0], pre.shape[1], 1 if dt == torch.bfloat16 else (2 if dt == torch.float16 else 0),
                              _native.stream_ptr())
        else:
            if b1 is not None:
                pre = pre + b1.to(dt)
            act = torch.relu(pre)
        out = act @ w2.t()
        if b2 is not None:
            out = out + b2.to(dt)
        ctx.save_for_backward(x2, w1, w2, pre, act)
        ctx.has_b = (b1 is not None, b2 is not None)
        ctx.mean = bias_grad_mean
        ctx.xshape = X.shape
        ctx.dtypes = (X.dtype, W1.dtype)
        return out.view(*X.shape[:-1], W2.shape[0])

    @staticmethod
    def backward(ctx, g):
        x2, w1, w2, pre, act = ctx.saved_tensors
        g2 = _flat2(g).to(act.dtype)
        rows = g2.shape[0]
        gW2 = g2.t() @ act
        gact = g2 @ w2
        gb2 = None
        if ctx.has_b[1]:
            gb2 = g2.float().sum(0, keepdim=True)
        nat = _native.load() if _native.use_native(g) else None
        if nat is not None and hasattr(nat, "relu_bwd_colsum") and gact.is_contiguous():
            gpre = torch.empty_like(gact)
            gb1 = torch.zeros(1, gact.shape[1], device=g.device, dtype=torch.float32)
            nat.relu_bwd_colsum(gact.data_ptr(), pre.data_ptr(), gpre.data_ptr(), gb1.data_ptr(),
                                rows, gact.shape[1], 1 if gact.dtype == torch.bfloat16 else (2 if gact.dtype == torch.float16 else 0),
                                _native.stream_ptr())
        else:
            gpre = gact * (pre > 0).to(gact.dtype)
            gb1 = gpre.float().sum(0, keepdim=True)
        if not ctx.has_b[0]:
            gb1 = None
        if ctx.mean:
            gb1 = gb1 / rows if gb1 is not None else None
            gb2 = gb2 / rows if gb2 is not None else None
        gW1 = gpre.t() @ x2
        gX = gpre @ w1
        xdt, wdt = ctx.dtypes
        cast = lambda t: None if t is None else t.to(wdt)  # noqa: E731
        return (gX.to(xdt).view(ctx.xshape), cast(gW1), cast(gb1), cast(gW2), cast(gb2), None)


def fused_mlp(X, W1, b1, W2, b2, bias_grad_mean=False):
    return FusedMLPFunction.apply(X, W1, b1, W2, b2, bias_grad_mean)
