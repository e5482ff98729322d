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
    """``packed`` (k = v = None): q is the fused projection output [B, L, 3, H, D] and the
    backward writes dq/dk/dv straight into one [B, L, 3, H, D] gradient (the kernels take
    its row stride) -- no stack/cat of three gradients (measured 77 us per layer at
    bs 256 x L 128 as a separate copy kernel)."""

    @staticmethod
    def forward(ctx, q, k, v, mask_u8, dropout_p: float, fill: float):
        nat = _native.native()
        packed = k is None
        qkv = q
        if packed:
            q, k, v = qkv.unbind(2)
        B, L, H, D = q.shape
        out = torch.empty(B, L, H, D, device=q.device, dtype=torch.bfloat16)
        lse = torch.empty(B, H, L, device=q.device, dtype=torch.float32)
        seed = int(torch.randint(0, 2**62, (1,)).item()) if dropout_p > 0 else 0
        sptr = DEVICE_SEED.data_ptr() if (DEVICE_SEED is not None and dropout_p > 0) else 0
        nat.attn_fwd(q.data_ptr(), k.data_ptr(), v.data_ptr(), _strides(q, k, v), out.data_ptr(), lse.data_ptr(),
                     0 if mask_u8 is None else mask_u8.data_ptr(), B, L, H, float(fill), float(dropout_p), seed,
                     sptr, _native.stream_ptr())
        ctx.save_for_backward(qkv if packed else q, None if packed else k, None if packed else v, out, lse, mask_u8)
        ctx.cfg = (float(fill), float(dropout_p), seed, sptr, packed)
        return out

    @staticmethod
    def backward(ctx, g):
        nat = _native.native()
        q, k, v, out, lse, mask_u8 = ctx.saved_tensors
        fill, p, seed, sptr, packed = ctx.cfg
        if packed:
            q, k, v = q.unbind(2)
        B, L, H, D = q.shape
        g = g.contiguous().to(torch.bfloat16)
        if packed:
            dqkv = torch.empty(B, L, 3, H, D, device=q.device, dtype=torch.bfloat16)
            dq, dk, dv = dqkv.unbind(2)
        else:
            dq = torch.empty(B, L, H, D, device=q.device, dtype=torch.bfloat16)
            dk = torch.empty_like(dq)
            dv = torch.empty_like(dq)
        delta = torch.empty(B, H, L, device=q.device, dtype=torch.float32)
        nat.attn_bwd(q.data_ptr(), k.data_ptr(), v.data_ptr(), _strides(q, k, v), out.data_ptr(), g.data_ptr(),
                     lse.data_ptr(), delta.data_ptr(), 0 if mask_u8 is None else mask_u8.data_ptr(),
                     dq.data_ptr(), dk.data_ptr(), dv.data_ptr(), B, L, H, fill, p, seed, sptr,
                     dq.stride(1) if packed else 0, _native.stream_ptr())
        if packed:
            return dqkv, None, None, None, None, None
        return dq, dk, dv, None, None, None


def _mask_u8(mask):
    if mask is None:
        return None
    m = mask if mask.dtype == torch.uint8 else (mask != 0).to(torch.uint8)
    return m.contiguous()


def attention_packed(qkv, mask=None, dropout_p=0.0, mask_value=None):
    """qkv: (B, L, 3, H, 64) bf16 with contiguous head dim (the fused Q/K/V projection
    output); gradient returned in the same packed layout."""
    fill = float("-inf") if mask_value is None else float(mask_value)
    return FlashAttention.apply(qkv, None, None, _mask_u8(mask), float(dropout_p), fill)


def attention_native(q, k, v, mask=None, dropout_p=0.0, mask_value=None):
    """q, k, v: (B, L, H, 64) bf16; mask (B, L) with nonzero = keep; ``mask_value`` None =
    true masking, else the reference's fill value for masked scores."""
    fill = float("-inf") if mask_value is None else float(mask_value)
    return FlashAttention.apply(q, k, v, _mask_u8(mask), float(dropout_p), fill)
