"""Transformer position-wise FFN with its GEMM epilogues fused (reference
``transformer.py:159-177``: ``w_2(dropout(gelu(w_1(x))))``; survey K11).

Unfused, one FFN costs per step: GEMM ``x W_1^T + b_1`` -> a separate GELU-dropout pass (read
``a``, write ``h``) -> GEMM ``h W_2^T``; backward: GEMM ``g W_2`` (write ``dL/dh``) -> a
GELU-dropout backward pass (read ``dL/dh`` and ``a``, write ``ga``) -> a column-sum pass over
``ga`` for ``b_1``'s gradient.  Here the two ``W_1``-side activation passes live in GEMM
epilogues of the hand-written MFMA kernel (a token GEMM is a 1x1 convolution over the
tokens; ``csrc/kernels/conv_igemm_impl.h`` EPI_GELU_FWD / EPI_GELU_BWD):

* forward: one kernel stores ``a = x W_1^T + b_1`` (bf16, what backward differentiates GELU
  at) and ``h = dropout(gelu(a))``;
* backward: the data-gradient GEMM ``g_y W_2`` finishes through the GELU-dropout backward in
  its epilogue -- ``ga = keep * gelu'(a) * (g_y W_2) / (1 - p)`` leaves the kernel already,
  from the fp32 accumulator (``dL/dh`` is never rounded to bf16 or written) -- and the column
  sums of ``ga`` (``b_1``'s gradient) are reduced in the same epilogue (fp32 atomics).

The dropout mask is the counter hash of ``ops/dropout.py`` (same seed plumbing, so HIP-graph
replays draw fresh masks).  ``W_2``'s GEMMs and ``W_1``'s weight / input gradients stay
library GEMMs (hipBLASLt) or the split-K weight gradient of ``ops/linear.py``; parameters and
state-dict names are unchanged.
"""
from __future__ import annotations

import os

import torch
import torch.nn.functional as F

from . import _native
from .dropout import _seed
from .linear import bias_grad, bias_grad_into, cast_weight, direct_target, mark_ready, wgrad, wgrad_into

FUSED = os.environ.get("FDT_FFN_FUSED", "0") != "0"  # default set from the A/B below
# which side runs on the fused kernel: the forward epilogue GEMM replaces a 45 us library GEMM +
# a 46 us GELU-dropout pass with one ~76 us kernel, the backward one a library GEMM + the
# GELU-dropout-backward/column-sum pass; FDT_FFN_FUSED_SIDES = fwd | bwd | both
SIDES = os.environ.get("FDT_FFN_FUSED_SIDES", "both")
EPI_GELU_FWD, EPI_GELU_BWD = 5, 6
# (BM, BN, BK, kg) of the two fused GEMMs (tokens x d_ff, K = d_model): 128x128x32 (4 waves per
# SIMD) measured best at 32K tokens (scripts/bench_ffn.py: 76 / 80 us vs 96 / 99 at BK = 64)
TILE_FWD = (128, 128, 32, 1)
TILE_BWD = (128, 128, 32, 1)


def fusable(x: torch.Tensor, d_model: int, d_ff: int) -> bool:
    if not (FUSED and x.is_cuda and _native.use_native(x) and hasattr(_native.native(), "ffn_gemm")):
        return False
    dt = torch.get_autocast_dtype("cuda") if torch.is_autocast_enabled("cuda") else x.dtype
    return (dt == torch.bfloat16 and d_model >= 8 and (d_model & (d_model - 1)) == 0 and d_ff % 128 == 0
            and x.numel() // x.shape[-1] >= 4096)


def _gemm(x, w, out, epi, bias=None, out2=None, a_in=None, gb=None, p=0.0, seed=0, sptr=0, tile=TILE_FWD):
    M, K = x.shape
    N = w.shape[0]
    bm, bn, bk, kg = tile
    _native.native().ffn_gemm(x.data_ptr(), w.data_ptr(), out.data_ptr(), M, K, N, epi,
                              0 if bias is None else bias.data_ptr(), 0 if out2 is None else out2.data_ptr(),
                              0 if a_in is None else a_in.data_ptr(), 0 if gb is None else gb.data_ptr(),
                              float(p), int(seed), int(sptr), bm, bn, bk, kg, _native.stream_ptr())


class _FFNCore(torch.autograd.Function):
    """y = dropout(gelu(x W1^T + b1)) W2^T (+ b2) on bf16 operands; see the module docstring.
    ``out_bias_grad=False``: b2's gradient is left to the consumer of y (ops/dropout.py
    ``bias=``)."""

    @staticmethod
    def forward(ctx, x, w1, b1, w2, b2, p, out_bias_grad):
        dt = torch.bfloat16
        shp = x.shape
        x2 = x.reshape(-1, shp[-1]).to(dt).contiguous()
        w1c, w2c = cast_weight(w1, dt).contiguous(), cast_weight(w2, dt).contiguous()
        b1f = b1.detach().float().contiguous()
        M, d_ff = x2.shape[0], w1.shape[0]
        seed, sptr = _seed(p)
        if SIDES in ("both", "fwd"):
            a = torch.empty(M, d_ff, device=x.device, dtype=dt)
            h = torch.empty_like(a)
            _gemm(x2, w1c, a, EPI_GELU_FWD, bias=b1f, out2=h, p=p, seed=seed, sptr=sptr, tile=TILE_FWD)
        else:  # library GEMM + the standalone GELU-dropout pass (same mask: same seed, same hash)
            a = F.linear(x2, w1c, cast_weight(b1, dt))
            h = torch.empty_like(a)
            _native.native().gelu_dropout_fwd(a.data_ptr(), h.data_ptr(), a.numel(), float(p), seed, sptr,
                                              _native.stream_ptr())
        y = F.linear(h, w2c, None if b2 is None else cast_weight(b2, dt))
        ctx.save_for_backward(x2, a, h, w1c, w2c)
        ctx.cfg = (float(p), seed, sptr, bool(out_bias_grad), shp, x.dtype)
        ctx.params = (w1, b1, w2, b2)
        return y.view(*shp[:-1], w2.shape[0])

    @staticmethod
    def backward(ctx, gy):
        x2, a, h, w1c, w2c = ctx.saved_tensors
        p, seed, sptr, out_bias_grad, shp, xdt = ctx.cfg
        w1, b1, w2, b2 = ctx.params
        g2 = gy.reshape(-1, gy.shape[-1]).to(torch.bfloat16).contiguous()
        dw1 = db1 = dw2 = db2 = None
        # W2 side (library / split-K GEMMs): dW2 = g^T h, db2 = colsum(g)
        if ctx.needs_input_grad[3]:
            tgt = direct_target(w2)
            if tgt is not None:
                wgrad_into(g2, h, tgt)
                mark_ready(w2)
            else:
                dw2 = wgrad(g2, h).to(w2.dtype)
        if b2 is not None and ctx.needs_input_grad[4] and out_bias_grad:
            tgt = direct_target(b2)
            if tgt is not None:
                bias_grad_into(g2, tgt)
                mark_ready(b2)
            else:
                db2 = bias_grad(g2).to(b2.dtype)
        # ga = GELU-dropout backward of g W2, and b1's gradient, in one kernel
        ga = torch.empty_like(a)
        tb1 = direct_target(b1) if ctx.needs_input_grad[2] else None
        gb = tb1 if tb1 is not None else torch.zeros(a.shape[1], device=a.device, dtype=torch.float32)
        if SIDES in ("both", "bwd"):
            w2t = w2c.t().contiguous()  # [d_ff][d_model]: the kernel's K-contiguous weight operand
            _gemm(g2, w2t, ga, EPI_GELU_BWD, a_in=a, gb=gb, p=p, seed=seed, sptr=sptr, tile=TILE_BWD)
        else:
            gh = g2 @ w2c
            _native.native().gelu_dropout_bwd_colsum(gh.data_ptr(), a.data_ptr(), ga.data_ptr(), gb.data_ptr(),
                                                     a.shape[0], a.shape[1], p, seed, sptr, _native.stream_ptr())
        if ctx.needs_input_grad[2]:
            if tb1 is not None:
                mark_ready(b1)
            else:
                db1 = gb.view_as(b1).to(b1.dtype)
        if ctx.needs_input_grad[1]:
            tgt = direct_target(w1)
            if tgt is not None:
                wgrad_into(ga, x2, tgt)
                mark_ready(w1)
            else:
                dw1 = wgrad(ga, x2).to(w1.dtype)
        dx = None
        if ctx.needs_input_grad[0]:
            dx = (ga @ w1c).view(shp).to(xdt)
        return dx, dw1, db1, dw2, db2, None, None


def ffn_core(x, w1, b1, w2, b2, p: float, training: bool, out_bias_grad: bool = True) -> torch.Tensor:
    """``linear(dropout(gelu(linear(x, w1, b1))), w2, b2)`` with the fused GEMM epilogues
    (callers check ``fusable`` first)."""
    p = float(p) if training else 0.0
    with torch.autocast("cuda", enabled=False):
        return _FFNCore.apply(x, w1, b1, w2, b2, p, out_bias_grad)
