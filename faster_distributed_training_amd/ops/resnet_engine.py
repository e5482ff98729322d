"""MI355X execution engine for the ResNet family (NHWC, bf16, HIP kernels).

Replaces the per-module eager graph of the reference (``resnet.py:72-113,201-227``:
~7 kernels + 3-4 activation passes per FusedConvBN forward, ~15 in backward, recomputed
conv) with a *lazy-normalisation* dataflow:

* every conv output ``y`` is stored raw (bf16, NHWC ``[N*H*W, C]``) together with a
  per-channel affine ``(s, t)`` computed from its batch statistics — FusedConvBN
  numerics (unbiased var, ``1/(sqrt(var)+eps)``) or BatchNorm2d numerics;
* the *consumer* applies ``act(y*s + t)`` when it loads its operand; the residual join
  ``act(y3*s3 + t3 + shortcut)`` is one pass;
* autograd sees three kinds of nodes — ``ConvUnit`` (conv + its output statistics),
  ``ResidualJoin`` and the head — and the BatchNorm backward falls out of the chain
  rule as two per-channel reductions produced by the consumer plus an affine
  correction ``g_y += alpha + beta*y`` applied by the producer (see
  ``csrc/kernels/bn_kernels.hip``).

Conv GEMMs: ``conv_backend='miopen'`` runs the GEMM part through PyTorch-ROCm's
convolution (MIOpen) on channels-last bf16; the normalisation/statistics/activation/
residual work is always in our HIP kernels.  Reductions are deterministic (partial slabs
reduced in fp64), no host synchronisation anywhere in forward or backward.
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import _native

ACT_NONE, ACT_RELU, ACT_CELU = 0, 1, 2
MODE_FCBN, MODE_BN_TRAIN, MODE_BN_EVAL = 0, 1, 2
BF16 = torch.bfloat16
DT = {torch.float32: 0, torch.bfloat16: 1, torch.float16: 2}


def _sp():
    return _native.stream_ptr()


def _p(t):
    return 0 if t is None else t.data_ptr()


def _nchw_view(x_nhwc):
    """(N,H,W,C) contiguous -> (N,C,H,W) channels-last view (no copy)."""
    return x_nhwc.permute(0, 3, 1, 2)


def _nhwc(y_nchw_cl):
    """channels-last (N,C,H,W) -> (N,H,W,C) contiguous view (copy only if needed)."""
    y = y_nchw_cl.permute(0, 2, 3, 1)
    return y if y.is_contiguous() else y.contiguous()


def act_affine(x, s, t, act, alpha, out_dtype=BF16):
    nat = _native.native()
    C = x.shape[-1]
    M = x.numel() // C
    out = torch.empty(x.shape, device=x.device, dtype=out_dtype)
    nat.act_affine_fwd(x.data_ptr(), _p(s), _p(t), out.data_ptr(), M, C, act, float(alpha), DT[x.dtype],
                       DT[out_dtype], _sp())
    return out


def batch_stats(y, mode, eps, momentum=0.1, gamma=None, beta=None, run_mean=None, run_var=None, nbt=None):
    """Per-channel statistics of y [.., C] -> (s, t, save_mean, save_aux)."""
    nat = _native.native()
    C = y.shape[-1]
    M = y.numel() // C
    f32 = dict(device=y.device, dtype=torch.float32)
    s = torch.empty(C, **f32)
    t = torch.empty(C, **f32)
    sm = torch.empty(C, **f32)
    sa = torch.empty(C, **f32)
    if mode == MODE_BN_EVAL:
        nat.stats_finalize(0, 0, C, float(M), mode, float(eps), float(momentum), _p(gamma), _p(beta), _p(run_mean),
                           _p(run_var), 0, s.data_ptr(), t.data_ptr(), sm.data_ptr(), sa.data_ptr(), _sp())
        return s, t, sm, sa
    nb = nat.stats_num_blocks(M, C)
    part = torch.empty(nb, 2, C, **f32)
    nat.channel_stats_partial(y.data_ptr(), part.data_ptr(), M, C, DT[y.dtype], _sp())
    nat.stats_finalize(part.data_ptr(), nb, C, float(M), mode, float(eps), float(momentum), _p(gamma), _p(beta),
                       _p(run_mean), _p(run_var), _p(nbt), s.data_ptr(), t.data_ptr(), sm.data_ptr(), sa.data_ptr(),
                       _sp())
    return s, t, sm, sa


class ConvUnitFn(torch.autograd.Function):
    """y = conv(act(x*s_in + t_in), W);  (s_out, t_out) = stats(y).

    Inputs: x raw NHWC bf16; s_in/t_in fp32 [Cin] or None; w fp32 parameter;
    gamma/beta (BatchNorm2d affine) or None.  Outputs: y (NHWC bf16), s_out, t_out."""

    @staticmethod
    def forward(ctx, x, s_in, t_in, w, gamma, beta, cfg):
        (act_in, alpha_in, stride, pad, mode, eps, momentum, run_mean, run_var, nbt) = cfg
        dt = x.dtype
        a = act_affine(x, s_in, t_in, act_in, alpha_in, dt) if (s_in is not None or act_in != ACT_NONE) else x
        wb = w.to(dtype=dt, memory_format=torch.channels_last)
        y = _nhwc(F.conv2d(_nchw_view(a), wb, None, stride, pad))
        s, t, sm, sa = batch_stats(y, mode, eps, momentum, gamma, beta, run_mean, run_var, nbt)
        ctx.save_for_backward(x, s_in, t_in, a, wb, y, sm, sa, gamma)
        ctx.cfg = cfg
        ctx.wshape = w.shape
        ctx.wdtype = w.dtype
        return y, s, t

    @staticmethod
    def backward(ctx, g_y, g_s, g_t):
        x, s_in, t_in, a, wb, y, sm, sa, gamma = ctx.saved_tensors
        (act_in, alpha_in, stride, pad, mode, eps, _m, _rm, _rv, _n) = ctx.cfg
        nat = _native.native()
        C = y.shape[-1]
        M = y.numel() // C
        f32 = dict(device=y.device, dtype=torch.float32)
        # 1) statistics backward -> affine correction of dL/dy (+ BatchNorm2d affine grads)
        alpha = torch.empty(C, **f32)
        beta = torch.empty(C, **f32)
        g_gamma = torch.empty(C, **f32) if mode != MODE_FCBN else None
        g_beta = torch.empty(C, **f32) if mode != MODE_FCBN else None
        nat.stats_bwd_coef(_p(g_s), _p(g_t), C, float(M), mode, float(eps), sm.data_ptr(), sa.data_ptr(), _p(gamma),
                           alpha.data_ptr(), beta.data_ptr(), _p(g_gamma), _p(g_beta), _sp())
        g_yt = torch.empty_like(y)
        nat.affine_fold(_p(g_y.contiguous() if g_y is not None else None), y.data_ptr(), alpha.data_ptr(),
                        beta.data_ptr(), g_yt.data_ptr(), M, C, DT[y.dtype], _sp())
        # 2) conv backward (dgrad + wgrad)
        need_x = ctx.needs_input_grad[0] or ctx.needs_input_grad[1] or ctx.needs_input_grad[2]
        g_a, g_w, _ = torch.ops.aten.convolution_backward(
            _nchw_view(g_yt), _nchw_view(a), wb, None, [stride, stride], [pad, pad], [1, 1], False, [0, 0], 1,
            [need_x, ctx.needs_input_grad[3], False])
        g_w = g_w.to(ctx.wdtype).contiguous() if g_w is not None else None
        g_x = g_sin = g_tin = None
        if need_x:
            g_a = _nhwc(g_a)
            if s_in is not None or act_in != ACT_NONE:
                Cin = x.shape[-1]
                Min = x.numel() // Cin
                nb = nat.stats_num_blocks(Min, Cin)
                part = torch.empty(nb, 2, Cin, **f32)
                g_x = torch.empty_like(x)
                ones = s_in if s_in is not None else torch.ones(Cin, **f32)
                zeros = t_in if t_in is not None else torch.zeros(Cin, **f32)
                nat.act_bwd_reduce(g_a.data_ptr(), x.data_ptr(), ones.data_ptr(), zeros.data_ptr(), g_x.data_ptr(),
                                   part.data_ptr(), Min, Cin, act_in, float(alpha_in), DT[x.dtype], _sp())
                if s_in is not None:
                    red = torch.empty(2, Cin, **f32)
                    nat.reduce_partials(part.data_ptr(), nb, 2, Cin, red.data_ptr(), _sp())
                    g_sin, g_tin = red[0], red[1]
            else:
                g_x = g_a
        return g_x, g_sin, g_tin, g_w, g_gamma, g_beta, None


class ResidualJoinFn(torch.autograd.Function):
    """out = act(ya*sa + ta + (yb*sb + tb  |  xid))"""

    @staticmethod
    def forward(ctx, ya, sa, ta, yb, sb, tb, xid, act, alpha):
        nat = _native.native()
        C = ya.shape[-1]
        M = ya.numel() // C
        out = torch.empty_like(ya)
        nat.residual_act_fwd(ya.data_ptr(), sa.data_ptr(), ta.data_ptr(), _p(yb), _p(sb), _p(tb), _p(xid),
                             out.data_ptr(), M, C, act, float(alpha), DT[ya.dtype], _sp())
        ctx.save_for_backward(out, ya, sa, yb, sb)
        ctx.act = (act, alpha)
        ctx.has_b = yb is not None
        return out

    @staticmethod
    def backward(ctx, g):
        out, ya, sa, yb, sb = ctx.saved_tensors
        act, alpha = ctx.act
        nat = _native.native()
        C = ya.shape[-1]
        M = ya.numel() // C
        g = g.contiguous()
        gya = torch.empty_like(ya)
        gyb = torch.empty_like(ya)
        nb = nat.stats_num_blocks(M, C)
        f32 = dict(device=ya.device, dtype=torch.float32)
        part = torch.empty(nb, 3, C, **f32)
        nat.residual_act_bwd(g.data_ptr(), out.data_ptr(), ya.data_ptr(), sa.data_ptr(), _p(yb), _p(sb),
                             gya.data_ptr(), gyb.data_ptr(), part.data_ptr(), M, C, act, float(alpha), DT[ya.dtype],
                             _sp())
        red = torch.empty(3, C, **f32)
        nat.reduce_partials(part.data_ptr(), nb, 3, C, red.data_ptr(), _sp())
        if ctx.has_b:
            return gya, red[0], red[1], gyb, red[2], red[1], None, None, None
        return gya, red[0], red[1], None, None, None, gyb, None, None


class Lazy:
    """A tensor whose consumer must apply act(raw*s + t) (s/t None = identity)."""
    __slots__ = ("raw", "s", "t", "act", "alpha")

    def __init__(self, raw, s=None, t=None, act=ACT_NONE, alpha=1.0):
        self.raw, self.s, self.t, self.act, self.alpha = raw, s, t, act, alpha


def _act_of(m):
    if isinstance(m, nn.ReLU):
        return ACT_RELU, 1.0
    if isinstance(m, nn.CELU):
        return ACT_CELU, float(m.alpha)
    return None


def _conv_unit(inp: Lazy, conv, bn, training):
    """Run one conv (+ its normalisation statistics) on a lazy input."""
    from ..models.resnet import FusedConvBN
    if isinstance(conv, FusedConvBN):
        w, stride, pad = conv.conv_weight, 1, conv.padding
        mode, eps, mom, gamma, beta, rm, rv, nbt = MODE_FCBN, conv.eps, 0.0, None, None, None, None, None
    else:
        assert isinstance(conv, nn.Conv2d) and isinstance(bn, nn.BatchNorm2d)
        w, stride, pad = conv.weight, conv.stride[0], conv.padding[0]
        use_batch = training or not bn.track_running_stats
        mode = MODE_BN_TRAIN if use_batch else MODE_BN_EVAL
        eps, gamma, beta = bn.eps, bn.weight, bn.bias
        mom = bn.momentum if bn.momentum is not None else 0.1
        track = training and bn.track_running_stats
        rm = bn.running_mean if (track or mode == MODE_BN_EVAL) else None
        rv = bn.running_var if (track or mode == MODE_BN_EVAL) else None
        nbt = bn.num_batches_tracked if track else None
    cfg = (inp.act, inp.alpha, stride, pad, mode, eps, mom, rm, rv, nbt)
    y, s, t = ConvUnitFn.apply(inp.raw, inp.s, inp.t, w, gamma, beta, cfg)
    return Lazy(y, s, t)


def _run_chain(seq: nn.Sequential, inp: Lazy, training) -> Lazy:
    mods = list(seq)
    cur = inp
    i = 0
    while i < len(mods):
        m = mods[i]
        a = _act_of(m)
        if a is not None:
            cur = Lazy(cur.raw, cur.s, cur.t, a[0], a[1])
            i += 1
            continue
        bn = None
        if isinstance(m, nn.Conv2d):
            bn = mods[i + 1]
            i += 1
        cur = _conv_unit(cur, m, bn, training)
        i += 1
    return cur


def _block(blk, x, training):
    """BottleNeck / BasicBlock on a materialised NHWC input x."""
    from ..models.resnet import BottleNeck
    res = _run_chain(blk.residual_function, Lazy(x), training)
    if len(blk.shortcut) > 0:
        sc = _run_chain(blk.shortcut, Lazy(x), training)
        yb, sb, tb, xid = sc.raw, sc.s, sc.t, None
    else:
        yb = sb = tb = None
        xid = x
    act, alpha = (ACT_RELU, 1.0) if isinstance(blk, BottleNeck) else (ACT_CELU, 0.075)
    return ResidualJoinFn.apply(res.raw, res.s, res.t, yb, sb, tb, xid, act, alpha)


def to_nhwc(x, dt=BF16):
    if x.dim() == 4 and x.is_contiguous(memory_format=torch.channels_last) and x.dtype == dt:
        return x.permute(0, 2, 3, 1)
    return x.permute(0, 2, 3, 1).contiguous().to(dt)


def resnet_engine_forward(model, x):
    """Forward of ``models.resnet.ResNet`` through the HIP engine.  ``x``: NCHW (any
    float dtype / memory format) or already-channels-last bf16."""
    training = model.training
    xh = to_nhwc(x, getattr(model, "engine_dtype", BF16))
    stem = _run_chain(nn.Sequential(model.conv1[0]), Lazy(xh), training)
    act = _act_of(model.conv1[1])
    h = act_affine_fn(stem, act)
    for stage in (model.conv2_x, model.conv3_x, model.conv4_x, model.conv5_x):
        for blk in stage:
            h = _block(blk, h, training)
    pooled = h.float().mean(dim=(1, 2))
    return model.fc(pooled)


class ActAffineFn(torch.autograd.Function):
    """Materialise act(y*s + t) (used once, for the stem output)."""

    @staticmethod
    def forward(ctx, y, s, t, act, alpha):
        out = act_affine(y, s, t, act, alpha, y.dtype)
        ctx.save_for_backward(y, s, t)
        ctx.a = (act, alpha)
        return out

    @staticmethod
    def backward(ctx, g):
        y, s, t = ctx.saved_tensors
        act, alpha = ctx.a
        nat = _native.native()
        C = y.shape[-1]
        M = y.numel() // C
        nb = nat.stats_num_blocks(M, C)
        f32 = dict(device=y.device, dtype=torch.float32)
        part = torch.empty(nb, 2, C, **f32)
        gx = torch.empty_like(y)
        nat.act_bwd_reduce(g.contiguous().data_ptr(), y.data_ptr(), s.data_ptr(), t.data_ptr(), gx.data_ptr(),
                           part.data_ptr(), M, C, act, float(alpha), DT[y.dtype], _sp())
        red = torch.empty(2, C, **f32)
        nat.reduce_partials(part.data_ptr(), nb, 2, C, red.data_ptr(), _sp())
        return gx, red[0], red[1], None, None


def act_affine_fn(lz: Lazy, act):
    a, alpha = act if act is not None else (ACT_NONE, 1.0)
    return ActAffineFn.apply(lz.raw, lz.s, lz.t, a, alpha)
