"""ResNet family with the CIFAR stem and the FusedConvBN "module fusion" trick.

Architecture and parameter names follow the reference exactly so checkpoints are
interchangeable (``resnet.py:147-313``; key schema in survey §2.8):

* ``conv1 = Sequential(FusedConvBN(3, 64, 3, padding=1), CELU(0.075))`` (``resnet.py:237-240``)
* stages ``conv2_x..conv5_x`` with strides 1, 2, 2, 2 (``resnet.py:243-246``)
* BottleNeck stride-1: 3 x FusedConvBN (1x1, 3x3, 1x1) with ReLU between
  (``resnet.py:210-216``); stride-2: FusedConvBN 1x1 -> Conv2d 3x3 s2 + BatchNorm2d + ReLU
  -> FusedConvBN 1x1 (``resnet.py:201-208``)
* shortcut ``Conv2d 1x1 (stride s) + BatchNorm2d`` when the shape changes (``resnet.py:220-224``)
* BasicBlock uses CELU(0.075) (``resnet.py:147-190``)

On MI355X the whole network body runs through ``ops/resnet_fused.py`` (NHWC bf16,
hand-written MFMA implicit-GEMM conv kernels with batch-norm statistics in the epilogue
and normalisation + activation fused into the consumer's operand load); the
``nn.Sequential`` structure below is the CPU/oracle path and defines the state_dict.
"""
from __future__ import annotations

import math

import torch
import torch.nn as nn

from ..ops import _native
from ..ops.conv_bn import conv_bn_reference


class FusedConvBN(nn.Module):
    """Conv2d (no bias) followed by batch-statistics normalisation without affine.

    Same constructor as the reference (``resnet.py:116-131``); ``exp_avg_factor`` is
    accepted and ignored exactly like the reference (no running statistics, survey Q1).
    Only ``stride == 1`` is supported, as in the reference (``resnet.py:120``).
    """

    def __init__(self, in_channels, out_channels, kernel_size, stride=1, padding=0,
                 exp_avg_factor=0.1, eps=1e-3, device=None, dtype=None):
        super().__init__()
        assert stride == 1
        factory_kwargs = {"device": device, "dtype": dtype}
        self.conv_weight = nn.Parameter(
            torch.empty(out_channels, in_channels, kernel_size, kernel_size, **factory_kwargs))
        self.num_features = out_channels
        self.in_channels = in_channels
        self.kernel_size = kernel_size
        self.eps = eps
        self.stride = stride
        self.padding = padding
        self.reset_parameters(in_channels, kernel_size)

    def forward(self, X):
        return conv_bn_reference(X, self.conv_weight, self.stride, self.padding, self.eps)

    def reset_parameters(self, in_channels, kernel_size) -> None:
        n = in_channels * kernel_size * kernel_size
        stdv = 1.0 / math.sqrt(n)
        with torch.no_grad():
            self.conv_weight.uniform_(-stdv, stdv)

    def extra_repr(self):
        return (f"{self.in_channels}, {self.num_features}, kernel_size={self.kernel_size}, "
                f"padding={self.padding}, eps={self.eps}")


class BasicBlock(nn.Module):
    """ResNet-18/34 block (``resnet.py:147-190``): CELU(0.075) activations."""
    expansion = 1

    def __init__(self, in_channels, out_channels, stride=1):
        super().__init__()
        if stride != 1:
            self.residual_function = nn.Sequential(
                nn.Conv2d(in_channels, out_channels, kernel_size=3, stride=stride, padding=1, bias=False),
                nn.BatchNorm2d(out_channels),
                nn.CELU(alpha=0.075, inplace=True),
                FusedConvBN(out_channels, out_channels * BasicBlock.expansion, kernel_size=3, padding=1),
            )
        else:
            self.residual_function = nn.Sequential(
                FusedConvBN(in_channels, out_channels, kernel_size=3, padding=1),
                nn.CELU(alpha=0.075, inplace=True),
                FusedConvBN(out_channels, out_channels * BasicBlock.expansion, kernel_size=3, padding=1),
            )
        self.shortcut = nn.Sequential()
        if stride != 1 or in_channels != BasicBlock.expansion * out_channels:
            self.shortcut = nn.Sequential(
                nn.Conv2d(in_channels, out_channels * BasicBlock.expansion, kernel_size=1, stride=stride, bias=False),
                nn.BatchNorm2d(out_channels * BasicBlock.expansion),
            )
        self.stride = stride

    def forward(self, x):
        return nn.functional.celu(self.residual_function(x) + self.shortcut(x), alpha=0.075)


class BottleNeck(nn.Module):
    """ResNet-50/101/152 block (``resnet.py:193-227``)."""
    expansion = 4

    def __init__(self, in_channels, out_channels, stride=1):
        super().__init__()
        if stride != 1:
            self.residual_function = nn.Sequential(
                FusedConvBN(in_channels, out_channels, kernel_size=1),
                nn.ReLU(inplace=True),
                nn.Conv2d(out_channels, out_channels, stride=stride, kernel_size=3, padding=1, bias=False),
                nn.BatchNorm2d(out_channels),
                nn.ReLU(inplace=True),
                FusedConvBN(out_channels, out_channels * BottleNeck.expansion, kernel_size=1),
            )
        else:
            self.residual_function = nn.Sequential(
                FusedConvBN(in_channels, out_channels, kernel_size=1),
                nn.ReLU(inplace=True),
                FusedConvBN(out_channels, out_channels, kernel_size=3, padding=1),
                nn.ReLU(inplace=True),
                FusedConvBN(out_channels, out_channels * BottleNeck.expansion, kernel_size=1),
            )
        self.shortcut = nn.Sequential()
        if stride != 1 or in_channels != out_channels * BottleNeck.expansion:
            self.shortcut = nn.Sequential(
                nn.Conv2d(in_channels, out_channels * BottleNeck.expansion, stride=stride, kernel_size=1, bias=False),
                nn.BatchNorm2d(out_channels * BottleNeck.expansion),
            )
        self.stride = stride

    def forward(self, x):
        return torch.relu(self.residual_function(x) + self.shortcut(x))


class ResNet(nn.Module):
    """CIFAR ResNet (``resnet.py:230-283``).

    ``fast_path``: ``None`` = automatic (HIP engine when the input is on the GPU and the
    native extension is enabled), ``True``/``False`` to force.
    """

    def __init__(self, block, num_block, num_classes=100):
        super().__init__()
        self.in_channels = 64
        self.conv1 = nn.Sequential(
            FusedConvBN(3, 64, kernel_size=3, padding=1),
            nn.CELU(alpha=0.075, inplace=True))
        self.conv2_x = self._make_layer(block, 64, num_block[0], 1)
        self.conv3_x = self._make_layer(block, 128, num_block[1], 2)
        self.conv4_x = self._make_layer(block, 256, num_block[2], 2)
        self.conv5_x = self._make_layer(block, 512, num_block[3], 2)
        self.avg_pool = nn.AdaptiveAvgPool2d((1, 1))
        self.fc = nn.Linear(512 * block.expansion, num_classes)
        self.block = block
        self.num_block = list(num_block)
        self.fast_path = None
        self._engine = None

    def _make_layer(self, block, out_channels, num_blocks, stride):
        strides = [stride] + [1] * (num_blocks - 1)
        layers = []
        for s in strides:
            layers.append(block(self.in_channels, out_channels, s))
            self.in_channels = out_channels * block.expansion
        return nn.Sequential(*layers)

    def use_fast_path(self, x: torch.Tensor) -> bool:
        if self.fast_path is None:
            return _native.use_native(x)
        return bool(self.fast_path) and x.is_cuda

    def forward(self, x):
        if self.use_fast_path(x):
            from ..ops.resnet_fused import resnet_engine_forward
            return resnet_engine_forward(self, x)
        return self.forward_reference(x)

    def forward_reference(self, x):
        out = self.conv1(x)
        out = self.conv2_x(out)
        out = self.conv3_x(out)
        out = self.conv4_x(out)
        out = self.conv5_x(out)
        out = self.avg_pool(out)
        out = out.view(out.size(0), -1)
        return self.fc(out)


def resnet18(num_classes=10):
    return ResNet(BasicBlock, [2, 2, 2, 2], num_classes=num_classes)


def resnet34(num_classes=10):
    return ResNet(BasicBlock, [3, 4, 6, 3], num_classes=num_classes)


def resnet50(num_classes=10):
    return ResNet(BottleNeck, [3, 4, 6, 3], num_classes=num_classes)


def resnet101(num_classes=10):
    return ResNet(BottleNeck, [3, 4, 23, 3], num_classes=num_classes)


def resnet152(num_classes=10):
    return ResNet(BottleNeck, [3, 8, 36, 3], num_classes=num_classes)


def flops_per_image(model: ResNet, hw: int = 32) -> float:
    """Forward FLOPs (2*MACs) of convs + fc for one ``hw x hw`` image (survey: 2.60 GFLOP
    for ResNet-50)."""
    total = 0.0
    h = hw
    hooks = []

    def conv_hook(mod, inp, out):
        nonlocal total
        w = mod.conv_weight if isinstance(mod, FusedConvBN) else mod.weight
        total += 2.0 * w.numel() * out.shape[-1] * out.shape[-2]

    for m in model.modules():
        if isinstance(m, (FusedConvBN, nn.Conv2d)):
            hooks.append(m.register_forward_hook(conv_hook))
    fp = model.fast_path
    model.fast_path = False
    with torch.no_grad():
        model.forward_reference(torch.zeros(1, 3, h, h))
    model.fast_path = fp
    for hk in hooks:
        hk.remove()
    total += 2.0 * model.fc.weight.numel()
    return total
