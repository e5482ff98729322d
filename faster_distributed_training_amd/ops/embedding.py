"""Summed token + position + segment embedding, scaled by sqrt(d_model)
(reference ``Embeddings.forward``, ``transformer.py:150-156``).

GPU: ``csrc/kernels/embedding.hip`` — one wave per token row gathers the three table rows
with 16-B loads and writes the fp32 sum (one pass instead of three gathers + two adds +
a scale); the backward scatters the row gradient into the three tables with float
atomics shaped as whole 256-B rows (MI355X atomics run at ~1.3 TB/s for that shape).
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from . import _native


class _GatherRows(torch.autograd.Function):
    """``F.embedding`` whose backward is a static-shape ``index_add_`` (atomic scatter-add).

    ATen's dense embedding backward sorts the indices and compacts them with a
    data-dependent-size unique / partition (rocprim ``partition_kernel``): its output size is
    only known on the device, so under HIP-graph capture the buffers are sized from a value
    read at capture time and a replay with other token ids writes past them -- the
    ``HSA_STATUS_ERROR_MEMORY_APERTURE_VIOLATION`` of the captured ``--no-native``
    transformer step (round-2 review 5a).  ``index_add_`` has no data-dependent shape, so
    the reference-op path is graph-safe (and ``parallel.graphs.capture_guard`` refuses the
    ATen op inside any capture)."""

    @staticmethod
    def forward(ctx, idx, w):
        ctx.save_for_backward(idx)
        ctx.shape = w.shape
        return F.embedding(idx, w)

    @staticmethod
    def backward(ctx, g):
        (idx,) = ctx.saved_tensors
        gw = torch.zeros(ctx.shape, device=g.device, dtype=g.dtype)
        gw.index_add_(0, idx.reshape(-1), g.reshape(-1, ctx.shape[1]))
        return None, gw


def embedding_sum_reference(ids, types, pos_ids, tok_w, pos_w, seg_w, scale):
    L = ids.size(1)
    pos = _GatherRows.apply(pos_ids[:L], pos_w).unsqueeze(0)
    seg = _GatherRows.apply(types[:, :L], seg_w)
    tok = _GatherRows.apply(ids.long(), tok_w.float() if tok_w.dtype != torch.float32 else tok_w)
    return (pos + tok + seg) * scale


class _EmbeddingNative(torch.autograd.Function):
    @staticmethod
    def forward(ctx, ids, types, pos_ids, tok_w, pos_w, seg_w, scale):
        nat = _native.native()
        B, L = ids.shape
        d = tok_w.shape[1]
        ids32 = ids.to(torch.int32).contiguous()
        ty32 = types[:, :L].to(torch.int32).contiguous()
        pos32 = pos_ids[:L].to(torch.int32).contiguous()
        out = torch.empty(B, L, d, device=ids.device, dtype=torch.float32)
        nat.embedding_fwd(ids32.data_ptr(), ty32.data_ptr(), pos32.data_ptr(), tok_w.data_ptr(),
                          pos_w.data_ptr(), seg_w.data_ptr(), out.data_ptr(), B, L, d, float(scale),
                          tok_w.shape[0], pos_w.shape[0], seg_w.shape[0], _native.stream_ptr())
        ctx.save_for_backward(ids32, ty32, pos32)
        ctx.params = (tok_w, pos_w, seg_w)
        ctx.shapes = (tok_w.shape, pos_w.shape, seg_w.shape)
        ctx.scale = scale
        return out

    @staticmethod
    def backward(ctx, g):
        nat = _native.native()
        ids32, ty32, pos32 = ctx.saved_tensors
        B, L = ids32.shape
        (vt, d), (vp, _), (vs, _) = ctx.shapes
        g = g.contiguous().float()
        # the kernels accumulate atomically: with direct gradients (ops/linear.py) they add
        # straight into the flat fp32 gradient views -- no zeroed 62 MB token-table scratch
        # and no separate accumulate pass over it
        from .linear import direct_target, mark_ready
        tg = [direct_target(p) for p in ctx.params]
        direct = all(t is not None for t in tg) and all(ctx.needs_input_grad[3:6])
        if direct:
            gt, gp, gs = tg
        else:
            gt = torch.zeros(vt, d, device=g.device, dtype=torch.float32)
            gp = torch.zeros(vp, d, device=g.device, dtype=torch.float32)
            gs = torch.zeros(vs, d, device=g.device, dtype=torch.float32)
        nat.embedding_bwd(g.data_ptr(), ids32.data_ptr(), ty32.data_ptr(), pos32.data_ptr(), gt.data_ptr(),
                          gp.data_ptr(), gs.data_ptr(), B, L, d, float(ctx.scale), vt, vp, vs,
                          _native.stream_ptr())
        if direct:
            for p in ctx.params:
                mark_ready(p)
            return None, None, None, None, None, None, None
        return None, None, None, gt, gp, gs, None


def embedding_sum(ids, types, pos_ids, tok_w, pos_w, seg_w, scale):
    if (_native.use_native(ids) and tok_w.dtype == torch.float32 and tok_w.shape[1] % 256 == 0
            and hasattr(_native.native(), "embedding_fwd")):
        return _EmbeddingNative.apply(ids, types, pos_ids, tok_w, pos_w, seg_w, scale)
    return embedding_sum_reference(ids, types, pos_ids, tok_w, pos_w, seg_w, scale)
