"""Mixup family (reference ``resnet50_test.py:355-457``, ``transformer.py:71-80``).

* ``mixup_data`` (A1): scalar lambda ~ Beta(alpha, alpha) drawn on the host (no device
  sync), ``lam*x + (1-lam)*x[perm]``.
* ``MetaMixup`` (A2): per-sample lambda = sigmoid(theta), theta ~ U(0,1).  The reference
  re-creates theta every step and never optimises it (survey Q3): ``learnable=False``
  reproduces that; ``learnable=True`` keeps one theta registered with the optimiser.
* ``AttentionMixup`` (A3): per-element lambda map with ||lambda_i||^2 sample weight.
* ``mixup_criterion`` / ``mixup_criterion_meta`` (K7): lambda-weighted cross entropy.
  The reference meta criterion broadcasts to (B,1,1,B) (Q4); that equals
  ``mean(lam) * CE_a + (1-mean(lam)) * CE_b`` which ``faithful=True`` computes; the fixed
  form is the per-sample weighted mean.

GPU: ``csrc/kernels/mixup.hip`` fuses the permuted gather and the interpolation
(forward) and, in backward, computes dx through the inverse permutation (a gather, no
atomics) plus the per-sample d(lambda) reduction; the mixup cross entropy is one kernel
producing the loss and d(logits) together.
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import _native

DT = {torch.float32: 0, torch.bfloat16: 1, torch.float16: 2}


def sample_lambda(alpha: float, generator: torch.Generator | None = None) -> float:
    if alpha > 0:
        # Beta(a,a) via two Gammas on the host: one scalar per step, no device sync.
        g1 = torch._standard_gamma(torch.tensor([alpha], dtype=torch.float64), generator=generator)
        g2 = torch._standard_gamma(torch.tensor([alpha], dtype=torch.float64), generator=generator)
        return float(g1 / (g1 + g2))
    return float(alpha)


def _lam_tensor(lam, x):
    """Normalise lambda to a per-sample fp32 vector (B,) or a full per-element map."""
    b = x.shape[0]
    if isinstance(lam, (float, int)):
        return torch.full((b,), float(lam), device=x.device, dtype=torch.float32), "scalar"
    if lam.numel() == b:
        return lam.reshape(b).float(), "sample"
    return lam, "element"


class _MixupNative(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, perm, lam_vec, lam_requires_grad):
        nat = _native.native()
        xc = x.contiguous()
        b = xc.shape[0]
        inner = xc.numel() // b
        out = torch.empty_like(xc)
        perm32 = perm.to(torch.int32).contiguous()
        nat.mixup_fwd(xc.data_ptr(), perm32.data_ptr(), lam_vec.data_ptr(), out.data_ptr(), b, inner,
                      DT[xc.dtype], _native.stream_ptr())
        ctx.save_for_backward(xc, perm32, lam_vec)
        ctx.lrg = lam_requires_grad
        return out

    @staticmethod
    def backward(ctx, g):
        nat = _native.native()
        xc, perm32, lam_vec = ctx.saved_tensors
        b = xc.shape[0]
        inner = xc.numel() // b
        g = g.contiguous()
        inv = torch.empty_like(perm32)
        inv[perm32.long()] = torch.arange(b, device=g.device, dtype=torch.int32)
        gx = torch.empty_like(xc)
        glam = torch.empty(b, device=g.device, dtype=torch.float32) if ctx.lrg else None
        nat.mixup_bwd(g.data_ptr(), xc.data_ptr(), perm32.data_ptr(), inv.data_ptr(), lam_vec.data_ptr(),
                      gx.data_ptr(), _native.ptr(glam), b, inner, DT[xc.dtype], _native.stream_ptr())
        return gx, None, glam, None


def padded_channels_last(x: torch.Tensor):
    """If x (N,C,H,W) is the channel-slice view of a zero-padded NHWC buffer (N,H,W,cp)
    — the layout the device CIFAR loader emits for the conv engine — return cp."""
    if x.dim() != 4:
        return None
    N, C, H, W = x.shape
    s = x.stride()
    if s[1] == 1 and s[3] >= C and s[2] == W * s[3] and s[0] == H * W * s[3]:
        return s[3]
    return None


def mixup_interpolate(x: torch.Tensor, perm: torch.Tensor, lam) -> torch.Tensor:
    """lam * x + (1 - lam) * x[perm]; lam scalar, (B,)-shaped, or full map."""
    lv, kind = _lam_tensor(lam, x)
    if kind != "element" and _native.use_native(x) and x.dtype in DT:
        lrg = bool(getattr(lam, "requires_grad", False))
        cp = padded_channels_last(x)
        if cp is not None:
            # mix the whole padded per-sample block (pad channels stay zero) and keep the layout
            N, C, H, W = x.shape
            base = torch.as_strided(x, (N, H * W * cp), (H * W * cp, 1))
            out = _MixupNative.apply(base, perm, lv, lrg)
            return torch.as_strided(out, (N, C, H, W), (H * W * cp, 1, W * cp, cp))
        return _MixupNative.apply(x, perm, lv, lrg)
    if kind == "scalar":
        return float(lam) * x + (1 - float(lam)) * x[perm]
    shape = (x.shape[0],) + (1,) * (x.dim() - 1) if kind == "sample" else x.shape
    lv = lv.reshape(shape).to(x.dtype)
    return lv * x + (1 - lv) * x[perm]


def mixup_data(x, y, alpha=0.99, intra_only=False, generator=None):
    """(mixed_x, y_a, y_b, lam) — reference ``mixup_data`` (``resnet50_test.py:355-376``).
    ``intra_only`` keeps same-label pairs unmixed (vectorised, no per-sample loop)."""
    lam = sample_lambda(alpha, generator)
    b = x.size(0)
    if (not intra_only and _native.use_native(x) and x.dtype in DT and 1 <= b <= 1024 and y.dtype == torch.int64
            and y.is_cuda and hasattr(_native.native(), "mixup_prep")):
        # one kernel: device permutation (seeded from the host generator, no sync), the
        # permuted labels and the lambda vector
        seed = int(torch.randint(0, 2**62, (1,), generator=generator).item())
        perm = torch.empty(b, device=x.device, dtype=torch.int32)
        yb = torch.empty(b, device=x.device, dtype=torch.int64)
        lv = torch.empty(b, device=x.device, dtype=torch.float32)
        yc = y.contiguous()
        _native.native().mixup_prep(yc.data_ptr(), b, float(lam), seed, perm.data_ptr(), yb.data_ptr(), lv.data_ptr(),
                                    _native.stream_ptr())
        return mixup_interpolate(x, perm, lv), y, yb, lam
    perm = torch.randperm(b, device=x.device)
    if intra_only:
        same = (y == y[perm]).float()
        lam_vec = same + (1 - same) * lam
        mixed = mixup_interpolate(x, perm, lam_vec)
    else:
        mixed = mixup_interpolate(x, perm, lam)
    return mixed, y, y[perm], lam


class MetaMixup(nn.Module):
    """Per-sample learnable-lambda mixup (A2, ``resnet50_test.py:388-401``)."""

    def __init__(self, batch_size, device=None, learnable=False):
        super().__init__()
        self.lam = nn.Parameter(torch.rand(batch_size, 1, 1, 1, device=device))
        with torch.no_grad():
            self.lam.clamp_(0.0, 1.0)
        self.lam.requires_grad_(learnable)
        self.batch_size = batch_size
        self.learnable = learnable

    def resample(self):
        """Faithful mode: fresh theta ~ U(0,1) every step (the reference re-instantiates)."""
        with torch.no_grad():
            self.lam.uniform_(0.0, 1.0)

    def forward(self, x, y):
        if not self.learnable:
            self.resample()
        b = x.size(0)
        perm = torch.randperm(b, device=x.device)
        lam = torch.sigmoid(self.lam[:b])
        mixed = mixup_interpolate(x, perm, lam.view(b))
        return mixed, y, y[perm], lam


class AttentionMixup(nn.Module):
    """Per-pixel lambda map (A3, ``resnet50_test.py:404-424``; defined but unused there)."""

    def __init__(self, batch_size, width, height, channel=3, device=None):
        super().__init__()
        self.lam = nn.Parameter(torch.rand(batch_size, channel, width, height, device=device))
        with torch.no_grad():
            self.lam.clamp_(0.0, 1.0)

    def forward(self, x, y):
        b = x.size(0)
        perm = torch.randperm(b, device=x.device)
        lam_attn = torch.sigmoid(self.lam[:b])
        mixed = lam_attn * x + (1 - lam_attn) * x[perm]
        lam_scale = (lam_attn.reshape(b, -1) ** 2).sum(1)
        return mixed, y, y[perm], lam_scale


# ----------------------------------------------------------------------------- losses

class _MixupCENative(torch.autograd.Function):
    """lam: per-sample fp32 vector (B,) or a python float (one lambda for the batch: no
    lambda vector, no d(lambda))."""

    @staticmethod
    def forward(ctx, logits, ya, yb, lam, weights_mean, meter_acc=None):
        nat = _native.native()
        ctx.out_dtype = logits.dtype
        # fp16 logits (loss-scaled training): d(logits) = (p - t)/B must be kept in fp32 until the
        # loss scale has multiplied it -- stored early in fp16, values below ~6e-5 would become
        # subnormal / zero and the scaler would no longer protect them.  The [B, classes]
        # upcast is negligible.  bf16 has fp32's exponent range and is stored directly.
        lg = (logits.float() if logits.dtype == torch.float16 else logits).contiguous()
        b, c = lg.shape
        loss = torch.empty((), device=lg.device, dtype=torch.float32)
        # d(logits) in the (compute) logits' dtype: the backward is one scaling kernel
        glog = torch.empty(b, c, device=lg.device, dtype=lg.dtype)
        vec = isinstance(lam, torch.Tensor)
        dlam = torch.empty(b, device=lg.device, dtype=torch.float32) if vec else None
        # int64 labels are read as they are; anything else as int32 copies (kept referenced
        # until the launch is enqueued: a temporary freed inside the argument list can be
        # recycled by the caching allocator for the second copy -- ya and yb would alias)
        l64 = ya.dtype == torch.int64 and yb.dtype == torch.int64
        lt = torch.int64 if l64 else torch.int32
        ya_c = ya.to(lt).contiguous()
        yb_c = yb.to(lt).contiguous()
        nat.mixup_ce_fwd(lg.data_ptr(), ya_c.data_ptr(), yb_c.data_ptr(), lam.data_ptr() if vec else 0,
                         0.0 if vec else float(lam), loss.data_ptr(), glog.data_ptr(), _native.ptr(dlam),
                         0 if meter_acc is None else meter_acc.data_ptr(), b, c, DT[lg.dtype], int(l64),
                         _native.stream_ptr())
        ctx.save_for_backward(glog, dlam)
        return loss

    @staticmethod
    def backward(ctx, gl):
        glog, dlam = ctx.saved_tensors
        glam = dlam * gl if (dlam is not None and ctx.needs_input_grad[3]) else None
        # (backward seeded with unit_grad(): d(loss) == 1 -- no scaling pass over d(logits))
        g = glog if getattr(gl, "_fdt_unit", False) else glog * gl  # (0-dim fp32 gl: stays in glog.dtype)
        if g.dtype != ctx.out_dtype:
            g = g.to(ctx.out_dtype)  # fp16: cast AFTER the loss scale is applied
        return g, None, None, glam, None, None


_UNIT: dict = {}


def unit_grad(device):
    """A persistent 0-dim fp32 one to seed ``loss.backward(unit_grad(dev))`` with: autograd
    hands the same tensor to the loss node, whose backward then skips its scaling pass (and
    autograd skips its ones_like fill) -- two launches per step."""
    t = _UNIT.get(device)
    if t is None:
        t = _UNIT[device] = torch.ones((), device=device, dtype=torch.float32)
        t._fdt_unit = True
    return t


def mixup_cross_entropy(logits, y_a, y_b, lam_vec, meter=None):
    """mean_i [lam_i CE(p_i, ya_i) + (1-lam_i) CE(p_i, yb_i)]; ``lam_vec`` (B,) or a float.
    ``meter`` (train.metrics.DeviceMeter): on the HIP path the same kernel also accumulates
    the step's loss / lambda-weighted accuracy into it (``meter.fused`` is then set)."""
    if (_native.use_native(logits) and logits.dim() == 2 and logits.shape[1] <= 1024
            and logits.dtype in DT and hasattr(_native.native(), "mixup_ce_fwd")):
        acc = None
        if meter is not None and getattr(meter, "acc", None) is not None and meter.acc.device == logits.device:
            acc = meter.acc
            meter.fused = True
        lam = lam_vec.float().contiguous() if isinstance(lam_vec, torch.Tensor) else float(lam_vec)
        return _MixupCENative.apply(logits, y_a, y_b, lam, False, acc)
    lf = logits.float()
    ce_a = F.cross_entropy(lf, y_a, reduction="none")
    ce_b = F.cross_entropy(lf, y_b, reduction="none")
    return (lam_vec * ce_a + (1 - lam_vec) * ce_b).mean()


def mixup_criterion(criterion, pred, y_a, y_b, lam, meter=None):
    """Scalar-lambda criterion (``resnet50_test.py:451-452``).  ``criterion`` is accepted
    for API parity; cross entropy is computed by the fused kernel."""
    if criterion is not None and not isinstance(criterion, nn.CrossEntropyLoss):
        return lam * criterion(pred, y_a) + (1 - lam) * criterion(pred, y_b)
    return mixup_cross_entropy(pred, y_a, y_b, float(lam), meter=meter)


def mixup_criterion_meta(criterion, pred, y_a, y_b, lam, faithful=False, meter=None):
    """Per-sample-lambda criterion (``resnet50_test.py:455-457``); see module doc (Q4)."""
    b = pred.shape[0]
    lv = lam.reshape(b).float()
    if faithful:
        lv = lv.mean().expand(b).contiguous()
    return mixup_cross_entropy(pred, y_a, y_b, lv, meter=meter)
