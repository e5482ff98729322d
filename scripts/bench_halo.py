#!/usr/bin/env python3
"""Stride-1 3x3 convs of ResNet-50 (CIFAR) at a batch: halo kernel (BN 64 / 128) vs the tuned
generic implicit-GEMM launch, forward (EPI_STATS) and data gradient (EPI_ACTBWD).
    python scripts/bench_halo.py --batch 1024"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from faster_distributed_training_amd.ops import conv_igemm as ci
from bench_conv import timeit

SHAPES = [(32, 64, 64), (16, 128, 128), (8, 256, 256), (4, 512, 512)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1024)
    a = ap.parse_args()
    dev = torch.device("cuda")
    N = a.batch
    nat = ci._native.native()
    for H, Cin, Cout in SHAPES:
        shp = ci.ConvShape(Cin, Cout, 3, 1, 1)
        x = torch.randn(N, H, H, Cin, device=dev).to(torch.bfloat16)
        w = torch.randn(Cout, Cin, 3, 3, device=dev) / (Cin * 9) ** 0.5
        wf, wd = ci.alloc_packed(shp, dev)
        ci.pack_weights([(w, wf, wd, shp)])
        g = torch.randn(N, H, H, Cout, device=dev).to(torch.bfloat16)
        es, et = torch.ones(Cin, device=dev), torch.zeros(Cin, device=dev)
        flops = 2.0 * N * H * H * Cin * Cout * 9
        res = []
        for halo in (False, 64, 128):
            if halo and (Cout % halo or not nat.conv3x3_halo_supported(N, H, H, Cin, Cout, halo)):
                res.append("   -   ")
                continue
            f = timeit(lambda: ci.conv_fwd(x, wf, shp, halo=halo), 10)
            d = timeit(lambda: ci.conv_dgrad(g, None, None, None, wd, shp, (N, H, H, Cin), epi=ci.EPI_ACTBWD, ex=x,
                                             es=es, et=et, act=1, halo=halo), 10)
            res.append(f"{f * 1e3:7.1f}/{d * 1e3:7.1f} us ({flops / f / 1e9:5.0f}/{flops / d / 1e9:5.0f} TF/s)")
        print(f"{H:3d}x{H:<3d} {Cin:4d}->{Cout:4d}  generic {res[0]}  halo64 {res[1]}  halo128 {res[2]}", flush=True)


if __name__ == "__main__":
    main()
