"""Conv + batch-statistics normalisation ("FusedConvBN"), reference semantics.

Reference: ``resnet.py:72-113`` (``FusedConvBN2DFunction``) and ``resnet.py:116-144``
(``FusedConvBN``).  Numerics that define the model and are kept exactly (survey Q1/Q2):

* batch statistics over (N, H, W) in train *and* eval mode, no affine, no running stats;
* **unbiased** variance and ``(y - mean) / (sqrt(var) + eps)`` with ``eps = 1e-3``.

This file holds the pure-PyTorch implementation (CPU path and numerics oracle).  The
MI355X path is the ResNet engine (``ops/resnet_fused.py`` driving the implicit-GEMM kernels
of ``ops/conv_igemm.py``), which fuses the normalisation into the HIP kernels; both compute
the same function.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F


def bn_stats_unbiased(y: torch.Tensor):
    """(mean, sqrt(unbiased var)) per channel of an NCHW tensor (fp32 math)."""
    yf = y.float()
    mean = yf.mean(dim=(0, 2, 3))
    var = yf.var(dim=(0, 2, 3), unbiased=True)
    return mean, var.sqrt()


def conv_bn_reference(x: torch.Tensor, w: torch.Tensor, stride: int = 1, padding: int = 0,
                      eps: float = 1e-3) -> torch.Tensor:
    """Differentiable composite: conv2d -> (y - mean) / (sqrt(var_unbiased) + eps)."""
    y = F.conv2d(x, w, stride=stride, padding=padding)
    dims = (0, 2, 3)
    mean = y.mean(dim=dims, keepdim=True)
    var = y.var(dim=dims, unbiased=True, keepdim=True)
    return (y - mean) / (var.sqrt() + eps)


class FusedConvBN2DFunction(torch.autograd.Function):
    """Hand-derived forward/backward with the reference's contract (saves only X and W,
    recomputes the conv in backward).  Used by the gradcheck parity tests and by the
    ``--faithful`` CPU path; ``ops/resnet_fused.py`` is the production GPU path."""

    @staticmethod
    def forward(ctx, X, W, stride=1, padding=1, eps=1e-3):
        assert X.ndim == 4
        ctx.stride, ctx.padding, ctx.eps = stride, padding, eps
        ctx.save_for_backward(X, W)
        y = F.conv2d(X, W, stride=stride, padding=padding)
        n = y.numel() // y.size(1)
        s = y.sum(dim=(0, 2, 3))
        sd = y.var(dim=(0, 2, 3), unbiased=True).sqrt()
        ctx.n, ctx.sum, ctx.sd = n, s, sd
        return (y - (s / n)[None, :, None, None]) / (sd + eps)[None, :, None, None]

    @staticmethod
    def backward(ctx, g):
        X, W = ctx.saved_tensors
        y = F.conv2d(X, W, stride=ctx.stride, padding=ctx.padding)
        gy = bn_backward_unbiased(g, y, ctx.sum / ctx.n, ctx.sd, ctx.n, ctx.eps)
        gx = torch.nn.grad.conv2d_input(X.shape, W, gy, stride=ctx.stride, padding=ctx.padding)
        gw = torch.nn.grad.conv2d_weight(X, W.shape, gy, stride=ctx.stride, padding=ctx.padding)
        return gx, gw, None, None, None


def bn_backward_unbiased(g, y, mean, sd, n, eps):
    """d/dy of z = (y - mean)/(sd + eps), sd = sqrt(sum((y-mean)^2)/(n-1)).

    dz_i/dy_j = s*(delta_ij - 1/n) - s^2 * (y_i - mean) * (y_j - mean) / ((n-1) * sd)
    with s = 1/(sd+eps); so  gy = s*(g - mean(g)) - s^2/((n-1) sd) * yc * sum(g*yc)."""
    r = lambda v: v[None, :, None, None]  # noqa: E731
    s = 1.0 / (sd + eps)
    yc = y - r(mean)
    sg = g.sum(dim=(0, 2, 3))
    sgy = (g * yc).sum(dim=(0, 2, 3))
    return r(s) * (g - r(sg / n)) - r(s * s * sgy / ((n - 1) * sd)) * yc
