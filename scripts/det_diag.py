#!/usr/bin/env python3
"""Numerics of the deterministic engine mode vs the default mode and the fp32 reference:
logit / gradient relative errors of (default, default), (det, det), (det, default) and of
each against the fp32 PyTorch model and its bf16-autocast run (one ResNet train step)."""
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, ".")
from faster_distributed_training_amd.models import resnet as R  # noqa: E402
from faster_distributed_training_amd.ops import _native  # noqa: E402


def rel(a, b):
    return ((a.float() - b.float()).norm() / (b.float().norm() + 1e-12)).item()


def run(arch, x, y, fast, det=False, autocast=False):
    _native.set_deterministic(det)
    torch.manual_seed(0)
    m = getattr(R, arch)(10).cuda()
    m.fast_path = fast
    m.graph_engine = False
    if autocast:
        with torch.autocast("cuda", dtype=torch.bfloat16):
            out = m(x)
    else:
        out = m(x)
    F.cross_entropy(out.float(), y).backward()
    torch.cuda.synchronize()
    g = torch.cat([p.grad.flatten().float() for p in m.parameters()])
    _native.set_deterministic(False)
    return out.detach().float(), g


def main():
    torch.backends.cudnn.allow_tf32 = False
    torch.backends.cuda.matmul.allow_tf32 = False
    for arch, bs, seed in (("resnet50", 64, 5), ("resnet50", 64, 1), ("resnet18", 16, 500)):
        gen = torch.Generator().manual_seed(seed)
        x = torch.randn(bs, 3, 32, 32, generator=gen).cuda()
        y = torch.randint(0, 10, (bs,), generator=gen).cuda()
        ref = run(arch, x, y, False)
        rbf = run(arch, x, y, False, autocast=True)
        d1, d2 = run(arch, x, y, True), run(arch, x, y, True)
        t1, t2 = run(arch, x, y, True, det=True), run(arch, x, y, True, det=True)
        print(f"{arch} bs{bs} seed{seed}")
        for name, (a, b) in {"bf16-autocast vs fp32": (rbf, ref), "default vs fp32": (d1, ref),
                             "det vs fp32": (t1, ref), "default vs default": (d2, d1),
                             "det vs det": (t2, t1), "det vs default": (t1, d1)}.items():
            print(f"  {name:24s} logits {rel(a[0], b[0]):.3e}  grads {rel(a[1], b[1]):.3e}")


if __name__ == "__main__":
    main()
