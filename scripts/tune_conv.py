#!/usr/bin/env python3
"""Tile sweep for the implicit-GEMM conv kernels on the ResNet-50 shapes.

For every (op, batch, shape) it times every legal (BM, BN, BK[, nsplit]) configuration on
the GPU (HIP events, random data) and writes the fastest into
``faster_distributed_training_amd/ops/conv_tuned.json`` — the table the engine consults
before falling back to ``conv_igemm.pick_tile``.

    python scripts/tune_conv.py --batches 1024 128 [--out path]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch

from faster_distributed_training_amd.ops import conv_igemm as ci
from bench_conv import SHAPES, timeit

FWD_TILES = [(128, 128, 64), (128, 64, 64), (64, 128, 64), (64, 64, 64), (256, 64, 64),
             (128, 128, 32), (128, 64, 32), (64, 128, 32), (64, 64, 32), (256, 128, 32),
             (64, 64, 128), (128, 64, 128), (64, 128, 128)]
WG_TILES = [(128, 128, 32), (64, 128, 32), (128, 64, 32), (64, 64, 32),
            (128, 128, 64), (64, 128, 64), (128, 64, 64), (64, 64, 64)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batches", type=int, nargs="+", default=[1024, 128])
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--max-m", type=int, default=0, help="only shapes with N*Ho*Wo <= this (0 = all)")
    ap.add_argument("--ksize", type=int, default=0, help="only kernels of this size (0 = all)")
    ap.add_argument("--ops", default="fwd,dgrad,wgrad", help="which ops to sweep")
    ap.add_argument("--splits", type=int, nargs="+", default=[1, 2, 4, 8],
                    help="split-K candidates for fwd/dgrad when the tile grid is small")
    ap.add_argument("--kg", type=int, nargs="+", default=[1, 2],
                    help="K-group candidates for fwd/dgrad (2: 8-wave workgroups, conv_igemm.KG_TILES, no split-K)")
    ap.add_argument("--base", default=None, help="table to start from (default: --out if it exists, else the "
                                                 "in-tree table)")
    ap.add_argument("--out", default=os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                                  "faster_distributed_training_amd", "ops", "conv_tuned.json"))
    a = ap.parse_args()
    dev = torch.device("cuda")
    table = {}
    base = a.base or (a.out if os.path.exists(a.out) else ci._TUNED_PATH)
    if os.path.exists(base):
        with open(base) as f:
            table = json.load(f)
    for N in a.batches:
        for (H, Cin, Cout, k, s, p, _cnt) in SHAPES:
            shp = ci.ConvShape(Cin, Cout, k, s, p)
            Ho0, Wo0 = ci.out_hw(H, H, shp)
            if a.max_m and N * Ho0 * Wo0 > a.max_m:
                continue
            if a.ksize and k != a.ksize:
                continue
            ops = set(a.ops.split(","))
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
            ex = torch.randn(N, H, H, Cin, device=dev).to(torch.bfloat16) if Cin >= 8 else None
            es = torch.ones(Cin, device=dev)
            et = torch.zeros(Cin, device=dev)
            gw = torch.empty(Cout, Cin, k, k, device=dev)
            key = ci.tune_key(N, H, shp)
            res = {}

            prev = table.get(key, {})

            def sweep(name, fn, tiles, legal, M, Nn):
                best = None
                for t in tiles:
                    if not legal(t):
                        continue
                    ntiles = -(-M // t[0]) * (Nn // t[1])
                    for ns in (a.splits if ntiles < 768 else [1]):
                        for kg in a.kg:
                            if kg == 2 and (ns != 1 or tuple(t) not in ci.KG_TILES):
                                continue
                            ms = timeit(lambda: fn(t, ns, kg), a.reps)
                            if best is None or ms < best[0]:
                                best = (ms, t, ns, kg)
                res[name] = dict(tile=best[1], nsplit=best[2], us=round(best[0] * 1e3, 1))
                if best[3] != 1:
                    res[name]["kg"] = best[3]

            # modes the fused engine actually launches (ops/resnet_fused.py): 3x3 convs get a
            # materialised input / pre-folded gradient; 1x1 convs fuse the transforms
            fwd_modes = ([0] if k > 1 else [0, 1]) if "fwd" in ops else []
            for pro in fwd_modes:
                sweep(f"fwd{pro}", lambda t, ns, kg: ci.conv_fwd(x, wf, shp, sv if pro else None, tv if pro else None,
                                                                  pro, 1.0, tile=t, nsplit=ns, kg=kg),
                      FWD_TILES, lambda t: Cout % t[1] == 0, N * Ho * Wo, Cout)
            if Cin >= 8 and "dgrad" in ops:
                dg = [(0, ci.EPI_ACTBWD)] if k > 1 else [(2, ci.EPI_ACTBWD), (2, ci.EPI_STORE)]
                for pro, epi in dg:
                    sweep(f"dgrad{pro}{epi}",
                          lambda t, ns, kg: ci.conv_dgrad(g, yy if pro else None, al if pro else None,
                                                          be if pro else None, wd, shp, (N, H, H, Cin), epi=epi,
                                                          ex=ex, es=es, et=et, act=1, tile=t, nsplit=ns, kg=kg),
                          FWD_TILES, lambda t: Cin % t[1] == 0, N * H * H // (s * s), Cin)
            ldw = shp.ntaps * shp.cxp
            slab = torch.empty(1024 * Cout * ldw // 4 + 1, device=dev)
            wg_modes = [(0, 0)] if k > 1 else [(1, 1), (1, 0)]
            if Cin < 8:
                wg_modes = [(1, 0)]
            if "wgrad" not in ops:
                wg_modes = []
            for fold, xaff in wg_modes:
                best = None
                for t in WG_TILES:
                    if Cout % t[0] or (t[1] == 128 and ldw < 128):
                        continue
                    tiles = (Cout // t[0]) * (-(-ldw // t[1]))
                    base = ci.wgrad_split(N * Ho * Wo, tiles)
                    for ns in sorted({max(1, base // 2), base, base * 2}):
                        if ns * Cout * ldw > slab.numel():
                            continue
                        ms = timeit(lambda: ci.conv_wgrad(g, yy if fold else None, al if fold else None,
                                                          be if fold else None, x, shp, gw, sv if xaff else None,
                                                          tv if xaff else None, xaff, tile=t, nsplit=ns, slab=slab),
                                    a.reps)
                        if best is None or ms < best[0]:
                            best = (ms, t, ns)
                res[f"wgrad{fold}{xaff}"] = dict(tile=best[1], nsplit=best[2], us=round(best[0] * 1e3, 1))
            prev.update(res)
            table[key] = prev
            print(key, json.dumps(res), flush=True)
            del x, g, yy, ex, slab
            torch.cuda.empty_cache()
    with open(a.out, "w") as f:
        json.dump(table, f, indent=1, sort_keys=True)
    print("wrote", a.out)


if __name__ == "__main__":
    main()
