#!/usr/bin/env python3
"""The 3x3 forward / data-gradient convolutions (prologue-free: materialised operands) with
their tuned launch vs the LDS-DMA ring of 3 buffers (kg 3) at several tiles -- the latency-bound small-M layers of the
8-GPU per-GPU batch and their batch-1024 counterparts.  Device time per call (graph replay of 20)
and the max abs difference to the tuned launch's output.

A 5-buffer ring (four K tiles in flight across the per-tile barrier) was built and measured with
this probe (profiles/r5/ring_probe_bs{128,1024}.txt, the "kg5" columns): slower than both the
register-staged loop and the 3-buffer ring on every shape and tile (e.g. 8x8 256->256 at batch
128, (64, 64, 64): 26.3 / 27.8 / 43.6 us for kg 1 / 3 / 5) -- deeper DMA prefetch only adds LDS
footprint (fewer resident workgroups) to layers that are latency- not bandwidth-bound -- so it
was not kept; the probe now covers kg 1 and 3."""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from faster_distributed_training_amd.ops import conv_igemm as ci  # noqa: E402
from roofline_layers import timeit  # noqa: E402

SHAPES = [(8, 256, 256), (16, 128, 128), (4, 512, 512), (32, 64, 64)]
TILES = [(64, 128, 64), (64, 64, 64), (128, 64, 64), (64, 128, 32), (128, 128, 32)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=128)
    a = ap.parse_args()
    dev = torch.device("cuda")
    torch.manual_seed(0)
    N = a.batch
    for (H, C, Co) in SHAPES:
        shp = ci.ConvShape(C, Co, 3, 1, 1)
        x = torch.randn(N, H, H, shp.cxp, device=dev).to(torch.bfloat16)
        w = torch.randn(Co, C, 3, 3, device=dev) / (C * 9) ** 0.5
        wf, wd = ci.alloc_packed(shp, dev, dgrad=True)
        ci.pack_weights([(w, wf, wd, shp)])
        g = (torch.randn(N, H, H, Co, device=dev) * 0.1).to(torch.bfloat16)
        ex = torch.randn(N, H, H, C, device=dev).to(torch.bfloat16)
        es, et = torch.ones(C, device=dev), torch.zeros(C, device=dev)
        part = ci.stat_slots(2, C, dev, N * H * H)
        fwd = lambda **kw: ci.conv_fwd(x, wf, shp, **kw)[0]  # noqa: E731
        dgr = lambda **kw: ci.conv_dgrad(g, None, None, None, wd, shp, tuple(x.shape), epi=ci.EPI_ACTBWD,  # noqa: E731
                                         ex=ex, es=es, et=et, act=1, part=part, **kw)[0]
        for name, fn in (("fwd", fwd), ("dgrad", dgr)):
            ref = fn().float()
            res = [f"tuned {timeit(fn, 20) * 1e3:6.1f}"]
            for tile in TILES:
                if Co % tile[1] and name == "fwd" or C % tile[1] and name == "dgrad":
                    continue
                for kg in (1, 3):
                    try:
                        us = timeit(lambda: fn(tile=tile, nsplit=1, kg=kg), 20) * 1e3
                        err = (fn(tile=tile, nsplit=1, kg=kg).float() - ref).abs().max().item()
                    except Exception as e:  # noqa: BLE001 (LDS overflow etc.)
                        res.append(f"{tile}/kg{kg} {type(e).__name__}")
                        continue
                    res.append(f"{tile}/kg{kg} {us:6.1f}" + (f" (d {err:.1e})" if err > 0.05 else ""))
            print(f"N {N} {H}x{H} {C}->{Co} {name}: " + "  ".join(res), flush=True)


if __name__ == "__main__":
    main()
