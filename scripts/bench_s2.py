#!/usr/bin/env python3
"""The stride-2 3x3 data gradients of ResNet-50 (the first conv of stages 2-4's first blocks):
the 2- and 4-tap output-parity classes through the halo loop (conv_h3.hip, kg 6) against all four
classes on the implicit-GEMM kernel.  Device time per call under graph replay.

    python scripts/bench_s2.py --batch 1024
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from faster_distributed_training_amd.ops import conv_igemm as ci  # noqa: E402
from roofline_layers import timeit  # noqa: E402

SHAPES = [(32, 128, 128), (16, 256, 256), (8, 512, 512)]  # input H, Cin, Cout


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    dev = torch.device("cuda")
    N = a.batch
    for H, C, Co in SHAPES:
        shp = ci.ConvShape(C, Co, 3, 2, 1)
        w = torch.randn(Co, C, 3, 3, device=dev) / (C * 9) ** 0.5
        wf, wd = ci.alloc_packed(shp, dev)
        ci.pack_weights([(w, wf, wd, shp)])
        g = torch.randn(N, H // 2, H // 2, Co, device=dev).to(torch.bfloat16)
        ex = torch.randn(N, H, H, C, device=dev).to(torch.bfloat16)
        es = torch.rand(C, device=dev) + 0.5
        et = torch.randn(C, device=dev) * 0.3
        xs = (N, H, H, C)
        flop = 2.0 * N * (H // 2) ** 2 * Co * C * 9
        fn = lambda: ci.conv_dgrad(g, None, None, None, wd, shp, xs, epi=ci.EPI_ACTBWD, ex=ex, es=es, et=et,  # noqa
                                   act=1)[0]
        res = []
        outs = []
        for on in (False, True):
            ci.H3_S2 = on
            t = timeit(fn, a.reps)
            outs.append(fn().float())
            res.append(f"{'halo classes' if on else 'implicit GEMM'} {t * 1e3:6.1f} us ({flop / t / 1e9:5.0f} TF/s)")
        d = ((outs[1] - outs[0]).norm() / outs[0].norm()).item()
        print(f"N {N} {H}x{H} {C}->{Co} s2 dgrad: " + "  ".join(res) + f"  rel diff {d:.0e}", flush=True)


if __name__ == "__main__":
    main()
