#!/usr/bin/env python3
"""Per-shape microbenchmark: hand-written implicit-GEMM conv kernels vs MIOpen (PyTorch-ROCm
channels-last bf16) on every distinct ResNet-50 (CIFAR) convolution shape.

    python scripts/bench_conv.py --batch 1024 [--tile BMxBN] [--json out.json]

Times are device times from HIP events over R repetitions after warmup, same random
(normal) data for both implementations.  TF/s counts 2*M*N*K useful FLOPs.
"""
from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch
import torch.nn.functional as F

from faster_distributed_training_amd.ops import conv_igemm as ci

# (H, Cin, Cout, k, stride, pad, count in ResNet-50)
SHAPES = [
    (32, 3, 64, 3, 1, 1, 1),
    (32, 64, 64, 1, 1, 0, 1),
    (32, 64, 64, 3, 1, 1, 3),
    (32, 64, 256, 1, 1, 0, 4),
    (32, 256, 64, 1, 1, 0, 2),
    (32, 256, 128, 1, 1, 0, 1),
    (32, 128, 128, 3, 2, 1, 1),
    (16, 128, 512, 1, 1, 0, 4),
    (32, 256, 512, 1, 2, 0, 1),
    (16, 512, 128, 1, 1, 0, 3),
    (16, 128, 128, 3, 1, 1, 3),
    (16, 512, 256, 1, 1, 0, 1),
    (16, 256, 256, 3, 2, 1, 1),
    (8, 256, 1024, 1, 1, 0, 6),
    (16, 512, 1024, 1, 2, 0, 1),
    (8, 1024, 256, 1, 1, 0, 5),
    (8, 256, 256, 3, 1, 1, 5),
    (8, 1024, 512, 1, 1, 0, 1),
    (8, 512, 512, 3, 2, 1, 1),
    (4, 512, 2048, 1, 1, 0, 3),
    (8, 1024, 2048, 1, 2, 0, 1),
    (4, 2048, 512, 1, 1, 0, 2),
    (4, 512, 512, 3, 1, 1, 2),
]


def timeit(fn, reps=20, warm=3):
    for _ in range(warm):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--json", default=None)
    ap.add_argument("--tile", default=None)
    a = ap.parse_args()
    dev = torch.device("cuda")
    N = a.batch
    tile = tuple(int(v) for v in a.tile.split("x")) if a.tile else None
    rows = []
    tot = {"ours_fwd": 0, "ours_dgrad": 0, "ours_wgrad": 0, "miopen_fwd": 0, "miopen_dgrad": 0, "miopen_wgrad": 0}
    print(f"{'shape':34s} {'fwd us':>8s} {'miop':>8s} {'dgrad':>8s} {'miop':>8s} {'wgrad':>8s} {'miop':>8s}  TF/s(fwd ours/miop)")
    for (H, Cin, Cout, k, s, p, cnt) in SHAPES:
        shp = ci.ConvShape(Cin, Cout, k, s, p)
        torch.manual_seed(0)
        x = torch.randn(N, H, H, shp.cxp, device=dev).to(torch.bfloat16)
        w = torch.randn(Cout, Cin, k, k, device=dev) / (Cin * k * k) ** 0.5
        wf, wd = ci.alloc_packed(shp, dev, dgrad=Cin >= 8)
        ci.pack_weights([(w, wf, wd, shp)])
        Ho, Wo = ci.out_hw(H, H, shp)
        g = torch.randn(N, Ho, Wo, Cout, device=dev).to(torch.bfloat16)
        yy = torch.randn(N, Ho, Wo, Cout, device=dev).to(torch.bfloat16)
        al = torch.zeros(Cout, device=dev)
        be = torch.zeros(Cout, device=dev)
        sv = torch.ones(shp.cxp, device=dev)
        tv = torch.zeros(shp.cxp, device=dev)
        gw = torch.empty(Cout, Cin, k, k, device=dev)
        M = N * Ho * Wo
        flops = 2.0 * M * Cout * Cin * k * k

        t_f = timeit(lambda: ci.conv_fwd(x, wf, shp, sv, tv, 1, 1.0, tile=tile), a.reps)
        t_d = timeit(lambda: ci.conv_dgrad(g, yy, al, be, wd, shp, (N, H, H, Cin)), a.reps) if Cin >= 8 else float("nan")
        slab = torch.empty(64 * Cout * shp.ntaps * shp.cxp, device=dev)
        t_w = timeit(lambda: ci.conv_wgrad(g, yy, al, be, x, shp, gw, sv, tv, 1, slab=slab), a.reps)

        xc = x[..., :Cin].permute(0, 3, 1, 2)  # channels-last NCHW view
        if Cin != shp.cxp:
            xc = xc.contiguous(memory_format=torch.channels_last)
        wc = w.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        gc = g.permute(0, 3, 1, 2)
        t_mf = timeit(lambda: F.conv2d(xc, wc, None, s, p), a.reps)
        t_md = timeit(lambda: torch.ops.aten.convolution_backward(gc, xc, wc, None, [s, s], [p, p], [1, 1], False,
                                                                  [0, 0], 1, [True, False, False]), a.reps)
        t_mw = timeit(lambda: torch.ops.aten.convolution_backward(gc, xc, wc, None, [s, s], [p, p], [1, 1], False,
                                                                  [0, 0], 1, [False, True, False]), a.reps)
        r = dict(shape=f"{H}x{H} {Cin}->{Cout} k{k} s{s}", count=cnt, M=M, gflop=flops / 1e9,
                 ours_fwd=t_f * 1e3, miopen_fwd=t_mf * 1e3, ours_dgrad=t_d * 1e3, miopen_dgrad=t_md * 1e3,
                 ours_wgrad=t_w * 1e3, miopen_wgrad=t_mw * 1e3)
        rows.append(r)
        for key in tot:
            if r[key] == r[key]:
                tot[key] += r[key] * cnt
        print(f"{r['shape']:34s} {r['ours_fwd']:8.1f} {r['miopen_fwd']:8.1f} {r['ours_dgrad']:8.1f} "
              f"{r['miopen_dgrad']:8.1f} {r['ours_wgrad']:8.1f} {r['miopen_wgrad']:8.1f}  "
              f"{flops / t_f / 1e9:6.0f}/{flops / t_mf / 1e9:6.0f}", flush=True)
    print("network totals (us, weighted by layer count):", {k: round(v, 1) for k, v in tot.items()})
    if a.json:
        with open(a.json, "w") as f:
            json.dump(dict(batch=N, rows=rows, totals=tot), f, indent=1)


if __name__ == "__main__":
    main()
