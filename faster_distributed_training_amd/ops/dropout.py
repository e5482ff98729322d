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

``bias=``: the bias of the linear layer that produced the dropout input (the FFN's ``w_1`` /
``w_2``, the attention output projection).  Its gradient is the column sum of the gradient
these backward kernels store, so they accumulate it on the way (``*_bwd_colsum`` kernels:
fp32 atomics straight into the flat gradient view) and the linear skips its own column-sum
pass over the same tensor (``ops/linear.linear(..., bias_grad=False)``).
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


def _bias_dst(bias, cols, device):
    """(fp32 column-sum destination, direct?) for a fused bias gradient: the parameter's flat
    gradient view when the engine writes gradients directly (ops/linear.direct_target), else
    a zeroed buffer the backward returns."""
    from .linear import direct_target
    tgt = direct_target(bias)
    if tgt is not None and tgt.numel() == cols:
        return tgt, True
    return torch.zeros(cols, device=device, dtype=torch.float32), False


def _bias_done(bias, dst, direct):
    from .linear import mark_ready
    if direct:
        mark_ready(bias)
        return None
    return dst.view(bias.shape).to(bias.dtype)


class _DropoutAdd(torch.autograd.Function):
    @staticmethod
    def forward(ctx, y, x, p, res=None, bias=None):
        out = torch.empty_like(x)
        seed, sptr = _seed(p)
        _native.native().dropout_add_fwd(y.data_ptr(), x.data_ptr(), out.data_ptr(), y.numel(), float(p), seed, sptr,
                                         _native.stream_ptr())
        ctx.cfg = (float(p), seed, sptr, y.dtype)
        ctx.res = res
        ctx.bias = bias
        return out

    @staticmethod
    def backward(ctx, g):
        p, seed, sptr, ydt = ctx.cfg
        g = g.contiguous()
        if g.dtype != torch.float32:
            g = g.float()
        gy = torch.empty(g.shape, device=g.device, dtype=torch.bfloat16)
        db = None
        if ctx.bias is not None and ctx.needs_input_grad[4]:
            cols = g.shape[-1]
            dst, direct = _bias_dst(ctx.bias, cols, g.device)
            _native.native().dropout_bwd_colsum(g.data_ptr(), gy.data_ptr(), dst.data_ptr(), g.numel() // cols, cols,
                                                p, seed, sptr, _native.stream_ptr())
            db = _bias_done(ctx.bias, dst, direct)
        else:
            _native.native().dropout_bwd(g.data_ptr(), gy.data_ptr(), g.numel(), p, seed, sptr, _native.stream_ptr())
        if ctx.res is not None:  # the sublayer's LayerNorm backward adds the skip gradient
            ctx.res.g = g
            return gy.to(ydt), None, None, None, db
        return gy.to(ydt), g, None, None, db


class _GeluDropout(torch.autograd.Function):
    @staticmethod
    def forward(ctx, a, p, bias=None):
        h = torch.empty_like(a)
        seed, sptr = _seed(p)
        _native.native().gelu_dropout_fwd(a.data_ptr(), h.data_ptr(), a.numel(), float(p), seed, sptr,
                                          _native.stream_ptr())
        ctx.save_for_backward(a)
        ctx.cfg = (float(p), seed, sptr)
        ctx.bias = bias
        return h

    @staticmethod
    def backward(ctx, g):
        (a,) = ctx.saved_tensors
        p, seed, sptr = ctx.cfg
        g = g.contiguous().to(torch.bfloat16)
        ga = torch.empty_like(a)
        db = None
        if ctx.bias is not None and ctx.needs_input_grad[2]:
            cols = a.shape[-1]
            dst, direct = _bias_dst(ctx.bias, cols, a.device)
            _native.native().gelu_dropout_bwd_colsum(g.data_ptr(), a.data_ptr(), ga.data_ptr(), dst.data_ptr(),
                                                     a.numel() // cols, cols, p, seed, sptr, _native.stream_ptr())
            db = _bias_done(ctx.bias, dst, direct)
        else:
            _native.native().gelu_dropout_bwd(g.data_ptr(), a.data_ptr(), ga.data_ptr(), a.numel(), p, seed, sptr,
                                              _native.stream_ptr())
        return ga, None, db


class _BiasGradTap(torch.autograd.Function):
    """Identity on y whose backward also returns the bias gradient (column sums of dL/dy): the
    plain-PyTorch path of ``bias=`` (the linear that produced y skipped its bias gradient)."""

    @staticmethod
    def forward(ctx, y, bias):
        ctx.bshape, ctx.bdt = bias.shape, bias.dtype
        return y.view_as(y)

    @staticmethod
    def backward(ctx, g):
        db = g.reshape(-1, g.shape[-1]).sum(0, dtype=torch.float32)
        return g, db.view(ctx.bshape).to(ctx.bdt)


def _ok(t) -> bool:
    return (t.is_cuda and t.is_contiguous() and t.numel() % 8 == 0 and t.data_ptr() % 16 == 0
            and _native.use_native(t) and hasattr(_native.native(), "dropout_add_fwd"))


def _tap(y, bias):
    if bias is not None and bias.requires_grad and torch.is_grad_enabled():
        return _BiasGradTap.apply(y, bias)
    return y


def dropout_add(y: torch.Tensor, x: torch.Tensor, p: float, training: bool = True, res=None,
                bias=None) -> torch.Tensor:
    """``x + dropout(y, p)``.  ``res``: the ops/layernorm.ResidualGrad of the LayerNorm that
    consumed x (armed by its native forward): x's skip gradient is handed to that LayerNorm's
    backward instead of being summed by autograd.  ``bias``: see the module docstring (the
    producer of y was called with ``bias_grad=False``)."""
    p = float(p) if training else 0.0
    if _ok(y) and _ok(x) and y.dtype == torch.bfloat16 and x.dtype == torch.float32 and y.shape == x.shape:
        if bias is not None and (y.shape[-1] % 8 or bias.numel() != y.shape[-1]):
            y, bias = _tap(y, bias), None
        return _DropoutAdd.apply(y, x, p, res if (res is not None and res.armed) else None, bias)
    return F.dropout(_tap(y, bias), p, training) + x


def gelu_dropout(a: torch.Tensor, p: float, training: bool = True, bias=None) -> torch.Tensor:
    """``dropout(gelu(a), p)`` (exact erf GELU).  ``bias``: as in ``dropout_add``."""
    p = float(p) if training else 0.0
    if _ok(a) and a.dtype == torch.bfloat16:
        if bias is not None and (a.shape[-1] % 8 or bias.numel() != a.shape[-1]):
            a, bias = _tap(a, bias), None
        return _GeluDropout.apply(a, p, bias)
    return F.dropout(F.gelu(_tap(a, bias)), p, training)
