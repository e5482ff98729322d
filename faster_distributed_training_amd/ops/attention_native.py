"""Autograd wrapper of the fused HIP attention kernels (``csrc/kernels/attention.hip``).

q, k, v: (B, L, H, 64) bf16 with the head dim contiguous (the strided per-head views of
the Q/K/V projection outputs: no transpose copies).  Output (B, L, H, 64) contiguous.
Backward recomputes the probabilities from the saved log2-domain log-sum-exp; dropout is
regenerated from a per-call seed (counter-based hash), so no mask tensor is stored.
"""
from __future__ import annotations

import torch

from . import _native

HEAD_DIM = 64

# Set by a HIP-graph runner while it captures (train/graphs.py): a device uint64 re-drawn
# before every replay and XORed into each call's (capture-time constant) dropout seed.
DEVICE_SEED = None


def _strides(*ts):
    out = []
    for t in ts:
        sb, sl, sh, sd = t.stride()
        assert sd == 1, "attention: head dim must be contiguous"
        out += [sb, sl, sh]
    return out


def supported(q, k, v) -> bool:
    return (q.is_cuda and q.dtype == torch.bfloat16 and k.dtype == q.dtype and v.dtype == q.dtype
            and q.dim() == 4 and q.shape[-1] == HEAD_DIM and q.shape == k.shape == v.shape
            and q.stride(-1) == 1 and k.stride(-1) == 1 and v.stride(-1) == 1)


class FlashAttention(torch.autograd.Function):
    @staticmethod
    def forward(ctx, q, k, v, mask_u8, dropout_p: float, fill: float):
        nat = _native.native()
        B, L, H, D = q.shape
        out = torch.empty(B, L, H, D, device=q.device, dtype=torch.bfloat16)
        lse = torch.empty(B, H, L, device=q.device, dtype=torch.float32)
        seed = int(torch.randint(0, 2**62, (1,)).item()) if dropout_p > 0 else 0
        sptr = DEVICE_SEED.data_ptr() if (DEVICE_SEED is not None and dropout_p > 0) else 0
        nat.attn_fwd(q.data_ptr(), k.data_ptr(), v.data_ptr(), _strides(q, k, v), out.data_ptr(), lse.data_ptr(),
                     0 if mask_u8 is None else mask_u8.data_ptr(), B, L, H, float(fill), float(dropout_p), seed,
                     sptr, _native.stream_ptr())
        ctx.save_for_backward(q, k, v, out, lse, mask_u8)
        ctx.cfg = (float(fill), float(dropout_p), seed, sptr)
        return out

    @staticmethod
    def backward(ctx, g):
        nat = _native.native()
        q, k, v, out, lse, mask_u8 = ctx.saved_tensors
        fill, p, seed, sptr = ctx.cfg
        B, L, H, D = q.shape
        g = g.contiguous().to(torch.bfloat16)
        dq = torch.empty(B, L, H, D, device=q.device, dtype=torch.bfloat16)
        dk = torch.empty_like(dq)
        dv = torch.empty_like(dq)
        delta = torch.empty(B, H, L, device=q.device, dtype=torch.float32)
        nat.attn_bwd(q.data_ptr(), k.data_ptr(), v.data_ptr(), _strides(q, k, v), out.data_ptr(), g.data_ptr(),
                     lse.data_ptr(), delta.data_ptr(), 0 if mask_u8 is None else mask_u8.data_ptr(),
                     dq.data_ptr(), dk.data_ptr(), dv.data_ptr(), B, L, H, fill, p, seed, sptr, _native.stream_ptr())
        return dq, dk, dv, None, None, None


def attention_native(q, k, v, mask=None, dropout_p=0.0, mask_value=None):
    """q, k, v: (B, L, H, 64) bf16; mask (B, L) with nonzero = keep; ``mask_value`` None =
    true masking, else the reference's fill value for masked scores."""
    m = None
    if mask is not None:
        m = mask if mask.dtype == torch.uint8 else (mask != 0).to(torch.uint8)
        m = m.contiguous()
    fill = float("-inf") if mask_value is None else float(mask_value)
    return FlashAttention.apply(q, k, v, m, float(dropout_p), fill)
