#!/usr/bin/env python3
"""The 3x3 stride-1 convolutions of ResNet-50 / CIFAR: the halo-staged loop (kg 5,
csrc/kernels/conv_h3.hip) against the tuned implicit-GEMM launch, forward (plain operand, BN
statistics epilogue) and data gradient (pre-folded gradient, ReLU activation-backward epilogue).
Device time per call under graph replay; max relative difference of the two outputs.

    python scripts/bench_h3.py --batch 1024
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from faster_distributed_training_amd.ops import conv_igemm as ci  # noqa: E402
from roofline_layers import timeit  # noqa: E402

SHAPES = [(32, 64, 64), (16, 128, 128), (8, 256, 256), (4, 512, 512)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--only", default=None, help="comma list of ops (wgrad,fwd,dgrad)")
    a = ap.parse_args()
    dev = torch.device("cuda")
    N = a.batch
    for H, C, Co in SHAPES:
        shp = ci.ConvShape(C, Co, 3, 1, 1)
        x = torch.randn(N, H, H, C, device=dev).to(torch.bfloat16)
        w = torch.randn(Co, C, 3, 3, device=dev) / (C * 9) ** 0.5
        wf, wd = ci.alloc_packed(shp, dev)
        ci.pack_weights([(w, wf, wd, shp)])
        g = torch.randn(N, H, H, Co, device=dev).to(torch.bfloat16)
        ex = torch.randn(N, H, H, C, device=dev).to(torch.bfloat16)
        es = torch.rand(C, device=dev) + 0.5
        et = torch.randn(C, device=dev) * 0.3
        flop = 2.0 * N * H * H * Co * C * 9
        part = ci.stat_slots(2, Co, dev, N * H * H)
        pd = ci.stat_slots(2, C, dev, N * H * H)
        out = torch.zeros(Co, C, 3, 3, device=dev)
        ops = {
            "wgrad": lambda kg: ci.conv_wgrad(g, None, None, None, x, shp, out, h3=kg is not None),
            "fwd": lambda kg: ci.conv_fwd(x, wf, shp, part=part, kg=kg)[0],
            "dgrad": lambda kg: ci.conv_dgrad(g, None, None, None, wd, shp, (N, H, H, C), epi=ci.EPI_ACTBWD, ex=ex,
                                              es=es, et=et, act=1, part=pd, kg=kg)[0],
        }
        for name, fn in ops.items():
            if a.only and name not in a.only.split(","):
                continue
            if name == "wgrad":
                plan = ci.wh3_plan(N, H, H, shp, C, force=True)
                t_old = timeit(lambda: fn(None), a.reps)
                y_old = fn(None).clone()
                t_new = timeit(lambda: fn(True), a.reps)
                y_new = fn(True).clone()
                d = ((y_new - y_old).norm() / y_old.norm()).item()
                print(f"N {N} {H}x{H} {C}->{Co} wgrad: implicit GEMM {t_old * 1e3:6.1f} us ({flop / t_old / 1e9:5.0f} TF/s)"
                      f"  halo {plan}: {t_new * 1e3:6.1f} us ({flop / t_new / 1e9:5.0f} TF/s, {d:.0e})", flush=True)
                continue
            h3 = ci.h3_tile(N, H, H, shp, ci.PRO_NONE, Co if name == "fwd" else C, force=True)
            ci.H3 = False
            t_old = timeit(lambda: fn(None), a.reps)
            y_old = fn(None).float()
            res = []
            for loop, kg in (("dma", 5), ("dma", 6), ("dma", 7), ("dma64", 6), ("dma64", 7), ("dma", 8)):
                if kg == 8 and (Co if name == "fwd" else C) % 128:
                    continue
                if h3 is None:
                    continue
                ci.H3_LOOP = loop
                t_new = timeit(lambda: fn(kg), a.reps)
                y_new = fn(kg).float()
                ci.H3_LOOP = "auto"
                d = ((y_new - y_old).norm() / y_old.norm()).item()
                res.append(f"kg{kg}/{'64' if loop == 'dma64' else '128'} {t_new * 1e3:6.1f} us "
                           f"({flop / t_new / 1e9:5.0f} TF/s, {d:.0e})")
            ci.H3 = True
            print(f"N {N} {H}x{H} {C}->{Co} {name:5s}: tuned {t_old * 1e3:6.1f} us ({flop / t_old / 1e9:5.0f} TF/s)"
                  f"  halo {h3}: " + "  ".join(res), flush=True)


if __name__ == "__main__":
    main()
