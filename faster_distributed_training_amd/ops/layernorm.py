"""LayerNorm with the reference's numerics (``transformer.py:230-242``):

    y = a * (x - mean) / (std_unbiased + eps) + b,   eps = 1e-6 added to the *std*.

GPU: one HIP kernel per direction (``csrc/kernels/layernorm.hip``): one row per wave
(d = 512 -> 8 elements per lane, one 16-B load for bf16), fp32 statistics; the output
is written directly in the autocast dtype (the residual stream may stay fp32, like the
reference where the embedding output is fp32); the backward fuses both row reductions
and writes per-block dgamma/dbeta partials (no atomics, deterministic).
"""
from __future__ import annotations

import torch

from . import _native

DT = {torch.float32: 0, torch.bfloat16: 1, torch.float16: 2}


def layer_norm_reference(x, a, b, eps=1e-6):
    mean = x.mean(-1, keepdim=True)
    std = x.std(-1, keepdim=True)
    return a * (x - mean) / (std + eps) + b


class ResidualGrad:
    """Hand-off of a residual block's skip-path gradient (``x + f(LN(x))``, the transformer
    sublayers): ``dropout_add``'s backward parks dL/d(out) here instead of returning it as
    x's gradient, and the LayerNorm backward adds it to its own dL/dx inside the kernel --
    autograd never sees two gradients for x, so no separate fp32 add pass over the residual
    stream.  ``armed`` is set by the native LayerNorm forward (only then may the skip
    gradient be parked)."""
    __slots__ = ("armed", "g")

    def __init__(self):
        self.armed = False
        self.g = None


class _LayerNormNative(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, a, b, eps, out_dtype, res=None):
        nat = _native.native()
        shape = x.shape
        d = shape[-1]
        x2 = x.reshape(-1, d)
        if not x2.is_contiguous():
            x2 = x2.contiguous()
        rows = x2.shape[0]
        y = torch.empty(rows, d, device=x.device, dtype=out_dtype)
        mean = torch.empty(rows, device=x.device, dtype=torch.float32)
        rstd = torch.empty(rows, device=x.device, dtype=torch.float32)
        nat.layernorm_fwd(x2.data_ptr(), a.data_ptr(), b.data_ptr(), y.data_ptr(), mean.data_ptr(),
                          rstd.data_ptr(), rows, d, float(eps), DT[x2.dtype], DT[out_dtype], DT[a.dtype],
                          _native.stream_ptr())
        ctx.save_for_backward(x2, a, mean, rstd)
        ctx.params = (a, b)
        ctx.shape = shape
        ctx.eps = eps
        ctx.res = res
        if res is not None:
            res.armed = True
        return y.view(*shape[:-1], d)

    @staticmethod
    def backward(ctx, gy):
        nat = _native.native()
        x2, a, mean, rstd = ctx.saved_tensors
        rows, d = x2.shape
        gy2 = gy.reshape(rows, d)
        if not gy2.is_contiguous():
            gy2 = gy2.contiguous()
        gx = torch.empty_like(x2)
        # ~8-16 rows per 4-wave block: enough workgroups to fill the chip at 32 samples / GPU
        # (4096 rows: 512 blocks; the old 32 rows per block left half the CUs idle)
        nblk = max(1, min(2048, (rows + 7) // 8))
        part = torch.empty(nblk, 2, d, device=x2.device, dtype=torch.float32)  # [block][gamma | beta][d]
        gres = None
        if ctx.res is not None and ctx.res.g is not None:
            gres = ctx.res.g.reshape(rows, d)
            assert gres.dtype == x2.dtype and gres.is_contiguous()
            ctx.res.g = None
        nat.layernorm_bwd(gy2.data_ptr(), x2.data_ptr(), a.data_ptr(), mean.data_ptr(), rstd.data_ptr(),
                          gx.data_ptr(), 0 if gres is None else gres.data_ptr(), part.data_ptr(), rows, d, nblk,
                          DT[gy2.dtype], DT[x2.dtype], DT[a.dtype], float(ctx.eps), _native.stream_ptr())
        from .linear import direct_target, mark_ready
        pa, pb = ctx.params
        ta = direct_target(pa) if ctx.needs_input_grad[1] else None
        tb = direct_target(pb) if ctx.needs_input_grad[2] else None
        if ta is not None and tb is not None:  # partials folded straight into the fp32 grads
            sp = _native.stream_ptr()
            if tb.data_ptr() == ta.data_ptr() + d * 4:
                # gamma / beta adjacent in the flat gradient (utils/flat.py flat_adjacent): one
                # pass over the [block][2][d] partials
                nat.slab_sum_acc(part.data_ptr(), ta.data_ptr(), nblk, 2 * d, 2 * d, sp)
            else:
                nat.slab_sum_acc(part.data_ptr(), ta.data_ptr(), nblk, 2 * d, d, sp)
                nat.slab_sum_acc(part.data_ptr() + d * 4, tb.data_ptr(), nblk, 2 * d, d, sp)
            mark_ready(pa)
            mark_ready(pb)
            return gx.view(ctx.shape), None, None, None, None, None
        ga, gb = part.sum(0).unbind(0)
        return gx.view(ctx.shape), ga.to(a.dtype), gb.to(a.dtype), None, None, None


def layer_norm_unbiased(x, a, b, eps=1e-6, res: ResidualGrad | None = None):
    """``res``: the residual block's skip-gradient hand-off (see ResidualGrad)."""
    if (_native.use_native(x) and x.shape[-1] % 64 == 0 and 64 <= x.shape[-1] <= 2048
            and x.dtype in DT and a.dtype == torch.float32):
        out_dtype = torch.get_autocast_dtype("cuda") if torch.is_autocast_enabled("cuda") else x.dtype
        return _LayerNormNative.apply(x, a, b, eps, out_dtype, res)
    return layer_norm_reference(x, a, b, eps)
