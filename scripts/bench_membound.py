#!/usr/bin/env python3
"""Memory-bound conv microbenchmark: the 1x1 convolutions of ResNet-50 whose cost is their
epilogue traffic, per tile config, with effective HBM bandwidth on the MINIMAL byte count.

    python scripts/bench_membound.py [--batch 1024] [--reps 20]

ops: fwd   = conv(act(x*s+t)) + BN statistics epilogue (block's expanding 1x1)
     store = plain conv, no prologue / statistics (the store-path ceiling)
     join  = dgrad of the block's first 1x1 + the previous block's residual-join backward
     add   = dgrad + accumulate (EPI_ADD)
     actb  = dgrad through the producer's lazy BN + act (EPI_ACTBWD)
"""
from __future__ import annotations

import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from faster_distributed_training_amd.ops import conv_igemm as ci

BF = torch.bfloat16
# (H, Cin, Cout) of 1x1 convs
SHAPES = [(32, 64, 256), (32, 256, 64), (16, 128, 512), (16, 512, 128), (8, 256, 1024), (8, 1024, 256),
          (4, 512, 2048), (4, 2048, 512)]
TILES = [None, (128, 128, 32), (128, 128, 64), (128, 64, 64), (64, 128, 64), (64, 64, 64), (256, 128, 32),
         (256, 64, 64)]


def timeit(fn, reps):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps * 1e3  # us


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--ops", default="fwd,store,join,add,actb")
    ap.add_argument("--shape", default=None, help="H,Cin,Cout: only this shape")
    ap.add_argument("--tile", default=None, help="BM,BN,BK: only this tile")
    a = ap.parse_args()
    shapes = [tuple(map(int, a.shape.split(",")))] if a.shape else SHAPES
    tiles = [tuple(map(int, a.tile.split(",")))] if a.tile else TILES
    dev = torch.device("cuda")
    N = a.batch
    ops = a.ops.split(",")
    for H, Cin, Cout in shapes:
        M = N * H * H
        shp = ci.ConvShape(Cin, Cout, 1, 1, 0)
        w = torch.randn(Cout, Cin, 1, 1, device=dev) / Cin ** 0.5
        wf, wd = ci.alloc_packed(shp, dev)
        ci.pack_weights([(w, wf, wd, shp)])
        x = torch.randn(N, H, H, Cin, device=dev).to(BF)
        s = torch.rand(Cin, device=dev) + 0.5
        t = torch.randn(Cin, device=dev) * 0.1
        g = torch.randn(N, H, H, Cout, device=dev).to(BF)
        y = torch.randn(N, H, H, Cout, device=dev).to(BF)
        al = torch.randn(Cout, device=dev) * 0.01
        be = torch.randn(Cout, device=dev) * 0.01
        out = torch.randn(N, H, H, Cin, device=dev).to(BF)
        ya = torch.randn(N, H, H, Cin, device=dev).to(BF)
        mask = torch.randint(0, 255, (M * Cin // 8,), device=dev, dtype=torch.uint8)
        es = torch.rand(Cin, device=dev) + 0.5
        et = torch.randn(Cin, device=dev) * 0.1
        part_f = ci.stat_slots(2, Cout, dev)
        part_a = ci.stat_slots(2, Cin, dev)
        part3 = ci.stat_slots(3, Cin, dev)
        for op in ops:
            if op == "fwd":
                nbytes = M * Cin * 2 + M * Cout * 2
                n_out = Cout
                fn = lambda tile: ci.conv_fwd(x, wf, shp, s, t, 1, 1.0, tile=tile, part=part_f)
            elif op == "join":
                nbytes = M * Cout * 2 * 2 + M * Cin * 2 * 3 + M * Cin // 8
                n_out = Cin
                fn = lambda tile: ci.conv_dgrad(g, y, al, be, wd, shp, (N, H, H, Cin), epi=ci.EPI_JOINBWD, out=out,
                                                ex=ya, part=part3, act=1, alpha=1.0, jmask=mask, tile=tile)
            elif op == "store":
                # plain 1x1 (dgrad form, no prologue / statistics): reads [M, Cout], writes [M, Cin]
                nbytes = M * Cout * 2 + M * Cin * 2
                n_out = Cin
                fn = lambda tile: ci.conv_dgrad(g, None, None, None, wd, shp, (N, H, H, Cin), epi=ci.EPI_STORE,
                                                tile=tile)
            elif op == "add":
                nbytes = M * Cout * 2 * 2 + M * Cin * 2 * 2
                n_out = Cin
                fn = lambda tile: ci.conv_dgrad(g, y, al, be, wd, shp, (N, H, H, Cin), epi=ci.EPI_ADD, out=out,
                                                tile=tile)
            else:
                nbytes = M * Cout * 2 * 2 + M * Cin * 2 * 2
                n_out = Cin
                fn = lambda tile: ci.conv_dgrad(g, y, al, be, wd, shp, (N, H, H, Cin), epi=ci.EPI_ACTBWD, out=out,
                                                ex=ya, es=es, et=et, act=1, part=part_a, tile=tile)
            res = []
            for tile in tiles:
                if tile is not None and n_out % tile[1]:
                    continue
                try:
                    us = timeit(lambda: fn(tile), a.reps)
                except Exception as e:  # noqa: BLE001
                    res.append(f"{tile}: ERR {str(e)[:40]}")
                    continue
                res.append(f"{'tuned' if tile is None else 'x'.join(map(str, tile))}:{us:.0f}us/{nbytes / us / 1e6:.2f}")
            print(f"{op:5s} H{H} {Cin}->{Cout} min {nbytes / 1e6:.0f} MB | " + "  ".join(res), flush=True)


if __name__ == "__main__":
    main()
