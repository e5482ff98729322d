"""Fused dropout epilogues of the transformer sublayers (``csrc/kernels/dropout.hip``).

* ``dropout_add(y, x, p)`` = ``x + dropout(y)`` -- the residual connection of both sublayers
  (reference ``transformer.py:246-262``: ``self.dropout(sublayer(x)) + x``), y in the autocast
  dtype (bf16), x / result the fp32 residual stream.
* ``gelu_dropout(a, p)`` = ``dropout(gelu(a))`` -- the FFN hidden activation
  (``transformer.py:159-177``).

One streaming HIP pass per direction; the keep mask is a counter-based hash of (seed, element)
regenerated in backward (no mask tensor).  The host seed is drawn from torch's CPU generator
(``torch.manual_seed`` reproduces it); while a HIP-graph runner captures, the per-replay device
word ``attention_native.DEVICE_SEED`` is XORed in so each replay draws fresh masks.
Elsewhere (CPU, fp32, odd shapes) the plain PyTorch composition runs.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from . import _native


def _seed(p):
    from . import attention_native as AN
    seed = int(torch.randint(0, 2**62, (1,)).item()) if p > 0 else 0
    sptr = AN.DEVICE_SEED.data_ptr() if (AN.DEVICE_SEED is not None and p > 0) else 0
    return seed, sptr


class _DropoutAdd(torch.autograd.Function):
    @staticmethod
    def forward(ctx, y, x, p, res=None):
        out = torch.empty_like(x)
        seed, sptr = _seed(p)
        _native.native().dropout_add_fwd(y.data_ptr(), x.data_ptr(), out.data_ptr(), y.numel(), float(p), seed, sptr,
                                         _native.stream_ptr())
        ctx.cfg = (float(p), seed, sptr, y.dtype)
        ctx.res = res
        return out

    @staticmethod
    def backward(ctx, g):
        p, seed, sptr, ydt = ctx.cfg
        g = g.contiguous()
        if g.dtype != torch.float32:
            g = g.float()
        gy = torch.empty(g.shape, device=g.device, dtype=torch.bfloat16)
        _native.native().dropout_bwd(g.data_ptr(), gy.data_ptr(), g.numel(), p, seed, sptr, _native.stream_ptr())
        if ctx.res is not None:  # the sublayer's LayerNorm backward adds the skip gradient
            ctx.res.g = g
            return gy.to(ydt), None, None, None
        return gy.to(ydt), g, None, None


class _GeluDropout(torch.autograd.Function):
    @staticmethod
    def forward(ctx, a, p):
        h = torch.empty_like(a)
        seed, sptr = _seed(p)
        _native.native().gelu_dropout_fwd(a.data_ptr(), h.data_ptr(), a.numel(), float(p), seed, sptr,
                                          _native.stream_ptr())
        ctx.save_for_backward(a)
        ctx.cfg = (float(p), seed, sptr)
        return h

    @staticmethod
    def backward(ctx, g):
        (a,) = ctx.saved_tensors
        p, seed, sptr = ctx.cfg
        g = g.contiguous().to(torch.bfloat16)
        ga = torch.empty_like(a)
        _native.native().gelu_dropout_bwd(g.data_ptr(), a.data_ptr(), ga.data_ptr(), a.numel(), p, seed, sptr,
                                          _native.stream_ptr())
        return ga, None


def _ok(t) -> bool:
    return (t.is_cuda and t.is_contiguous() and t.numel() % 8 == 0 and t.data_ptr() % 16 == 0
            and _native.use_native(t) and hasattr(_native.native(), "dropout_add_fwd"))


def dropout_add(y: torch.Tensor, x: torch.Tensor, p: float, training: bool = True, res=None) -> torch.Tensor:
    """``x + dropout(y, p)``.  ``res``: the ops/layernorm.ResidualGrad of the LayerNorm that
    consumed x (armed by its native forward): x's skip gradient is handed to that LayerNorm's
    backward instead of being summed by autograd."""
    p = float(p) if training else 0.0
    if _ok(y) and _ok(x) and y.dtype == torch.bfloat16 and x.dtype == torch.float32 and y.shape == x.shape:
        return _DropoutAdd.apply(y, x, p, res if (res is not None and res.armed) else None)
    return F.dropout(y, p, training) + x


def gelu_dropout(a: torch.Tensor, p: float, training: bool = True) -> torch.Tensor:
    """``dropout(gelu(a), p)`` (exact erf GELU)."""
    p = float(p) if training else 0.0
    if _ok(a) and a.dtype == torch.bfloat16:
        return _GeluDropout.apply(a, p)
    return F.dropout(F.gelu(a), p, training)
