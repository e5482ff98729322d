#!/usr/bin/env python3
"""Transformer linear weight gradients dW += gy^T x (fp32 accumulate) at the 8-GPU share
(B=32 -> 4096 / 8192 tokens): the current split-K library bmm + slab_sum_acc path
(ops/linear.py wgrad_into) vs the MFMA weight-gradient kernel of the conv engine as a 1x1
"convolution" over the tokens, whose splits add straight into the gradient with fp32 atomics
(conv_igemm.conv_wgrad direct mode), at several (tile, splits).  Device time per call (graph
replay of 20) and max relative error vs an fp32 reference."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from faster_distributed_training_amd.ops import conv_igemm as ci  # noqa: E402
from faster_distributed_training_amd.ops import linear as L  # noqa: E402
from roofline_layers import timeit  # noqa: E402

SHAPES = [(4096, 1536, 512), (4096, 512, 512), (4096, 1024, 512), (4096, 512, 1024),
          (8192, 1536, 512), (8192, 512, 1024)]
CANDS = [((64, 64, 64), 4), ((64, 64, 64), 8), ((64, 64, 64), 16), ((128, 64, 64), 8), ((64, 128, 64), 8),
         ((128, 128, 64), 8), ((128, 128, 64), 16), ((128, 128, 32), 16), ((64, 64, 32), 16), ((128, 128, 64), 32)]


def main():
    dev = torch.device("cuda")
    torch.manual_seed(0)
    for (M, O, K) in SHAPES:
        gy = (torch.randn(M, O, device=dev) * 0.1).to(torch.bfloat16)
        x = torch.randn(M, K, device=dev).to(torch.bfloat16)
        ref = gy.float().t() @ x.float()
        dst = torch.zeros(O, K, device=dev)
        t_cur = timeit(lambda: L.wgrad_into(gy, x, dst), 20) * 1e3
        dst.zero_()
        L.wgrad_into(gy, x, dst)
        e_cur = ((dst - ref).abs().max() / ref.abs().max()).item()
        res = [f"current {t_cur:6.1f}us (e {e_cur:.1e})"]
        shp = ci.ConvShape(K, O, 1, 1, 0)
        g4, x4 = gy.view(M, 1, 1, O), x.view(M, 1, 1, K)
        best = None
        for tile, ns in CANDS:
            if O % tile[0] or K % tile[1]:
                continue
            fn = lambda: ci.conv_wgrad(g4, None, None, None, x4, shp, dst, accumulate=True, tile=tile,  # noqa: E731
                                       nsplit=ns)
            try:
                us = timeit(fn, 20) * 1e3
            except Exception as ex:  # noqa: BLE001
                res.append(f"{tile}/{ns}: {type(ex).__name__}")
                continue
            dst.zero_()
            fn()
            e = ((dst - ref).abs().max() / ref.abs().max()).item()
            if best is None or us < best[0]:
                best = (us, tile, ns)
            res.append(f"{tile}/{ns} {us:6.1f} (e {e:.1e})")
        flops = 2 * M * O * K
        print(f"M {M} out {O} in {K}: " + "  ".join(res) + f"  || best {best[1]}/{best[2]} {best[0]:.1f}us "
              f"= {flops / best[0] / 1e6:.0f} TFLOP/s", flush=True)


if __name__ == "__main__":
    main()
