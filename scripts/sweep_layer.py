#!/usr/bin/env python3
"""Sweep the launch configurations of one conv op of one shape with HIP-graph timing (the
engine's replay conditions): every (tile, nsplit[, kg]) the kernels support.

    python scripts/sweep_layer.py --op wgrad --shape 8,256,256,3,1,1 --batch 1024
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from faster_distributed_training_amd.ops import conv_igemm as ci  # noqa: E402
from roofline_layers import timeit  # noqa: E402
from tune_conv import FWD_TILES, WG_TILES  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--op", default="wgrad")
    ap.add_argument("--shape", default="8,256,256,3,1,1")
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--splits", type=int, nargs="+", default=[1, 2, 4, 7, 8, 14, 28])
    a = ap.parse_args()
    H, Cin, Cout, k, s, p = map(int, a.shape.split(","))
    dev = torch.device("cuda")
    N = a.batch
    shp = ci.ConvShape(Cin, Cout, k, s, p)
    torch.manual_seed(0)
    x = torch.randn(N, H, H, shp.cxp, device=dev).to(torch.bfloat16)
    w = torch.randn(Cout, Cin, k, k, device=dev) / (Cin * k * k) ** 0.5
    wf, wd = ci.alloc_packed(shp, dev)
    ci.pack_weights([(w, wf, wd, shp)])
    Ho, Wo = ci.out_hw(H, H, shp)
    g = torch.randn(N, Ho, Wo, Cout, device=dev).to(torch.bfloat16)
    gw = torch.empty(Cout, Cin, k, k, device=dev)
    slab = torch.empty(64 * Cout * shp.ntaps * shp.cxp, device=dev)
    flops = 2.0 * N * Ho * Wo * Cout * Cin * k * k
    res = []
    tiles = WG_TILES if a.op == "wgrad" else FWD_TILES
    for t in tiles:
        for ns in a.splits:
            if a.op == "wgrad":
                if Cout % t[0]:
                    continue
                fn = lambda: ci.conv_wgrad(g, None, None, None, x, shp, gw, tile=t, nsplit=ns, slab=slab)  # noqa: E731
            elif a.op == "fwd":
                if Cout % t[1]:
                    continue
                fn = lambda: ci.conv_fwd(x, wf, shp, tile=t, nsplit=ns)  # noqa: E731
            else:
                if Cin % t[1]:
                    continue
                fn = lambda: ci.conv_dgrad(g, None, None, None, wd, shp, (N, H, H, Cin), tile=t, nsplit=ns)  # noqa: E731
            try:
                us = timeit(fn, 10) * 1e3
            except Exception as e:  # noqa: BLE001
                print(f"{t} ns {ns}: {type(e).__name__} {str(e)[:60]}", flush=True)
                continue
            res.append((us, t, ns))
            print(f"{a.op} {a.shape} b{N} tile {t} nsplit {ns:3d}: {us:8.1f} us  {flops / us / 1e6:6.1f} TF/s", flush=True)
    res.sort()
    print("best:", [(round(u, 1), t, n) for u, t, n in res[:5]], flush=True)


if __name__ == "__main__":
    main()
