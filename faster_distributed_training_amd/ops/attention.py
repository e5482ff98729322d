"""Scaled dot-product attention with key-padding mask and attention dropout
(reference ``ScaledDotProduct``, ``transformer.py:180-193``).

Reference numerics: ``softmax(q k^T / sqrt(d_k) masked_fill(mask == 0, fill)) -> dropout
-> @ v``.  The reference fill is ``-1e-9`` (a bug: nothing is masked, survey Q7); pass
``mask_value=-1e-9`` for that behaviour, default is a true mask.

GPU: ``csrc/kernels/attention.hip`` (wrapper ``ops/attention_native.py``) — flash-style
fused kernels for head_dim 64 (bf16 MFMA, online softmax, in-kernel counter-based
dropout, no L x L materialisation); backward recomputes P from the saved log-sum-exp.
"""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F

from . import _native


def attention_reference(q, k, v, mask=None, dropout_p=0.0, mask_value=None, training=True):
    """q, k, v: (B, L, H, D); mask: (B, L) with 1 = keep.  Returns (B, L, H, D)."""
    q, k, v = (t.transpose(1, 2) for t in (q, k, v))
    d = q.size(-1)
    scores = torch.matmul(q, k.transpose(-2, -1)) / math.sqrt(d)
    if mask is not None:
        fill = -1e9 if mask_value is None else mask_value
        if mask_value is None:
            fill = torch.finfo(scores.dtype).min
        scores = scores.masked_fill(mask[:, None, None, :] == 0, fill)
    p = F.softmax(scores.float(), dim=-1).to(q.dtype)
    if dropout_p > 0 and training:
        p = F.dropout(p, dropout_p)
    return torch.matmul(p, v).transpose(1, 2)


def scaled_dot_product_attention(q, k, v, mask=None, dropout_p=0.0, mask_value=None):
    """q, k, v: (B, L, H, D); mask (B, L) 1 = keep.  MI355X: the fused HIP kernels for
    bf16 head_dim 64 (the model's configuration under autocast); otherwise the PyTorch
    reference composition (CPU oracle, fp32 runs)."""
    if _native.use_native(q):
        from . import attention_native as an
        if an.supported(q, k, v):
            return an.attention_native(q, k, v, mask, dropout_p, mask_value)
    return attention_reference(q, k, v, mask, dropout_p, mask_value)


def packed_attention(qkv, mask=None, dropout_p=0.0, mask_value=None):
    """qkv: (B, L, 3, H, D), the fused Q/K/V projection output.  On MI355X the HIP kernels
    read Q/K/V in place and write the packed gradient; otherwise unbind + the reference."""
    if _native.use_native(qkv):
        from . import attention_native as an
        q, k, v = qkv.unbind(2)
        if an.supported(q, k, v):
            return an.attention_packed(qkv, mask, dropout_p, mask_value)
    q, k, v = qkv.unbind(2)
    return attention_reference(q, k, v, mask, dropout_p, mask_value)
