#!/usr/bin/env python3
"""Per-layer roofline of the ResNet-50 (CIFAR) convolutions at the tuned launch configs the
engine uses (ops/conv_tuned.json): measured device time of every (shape, op) against its
ALGORITHMIC minimum -- each operand read once, each result written once, FLOPs at the dense
bf16 MFMA peak -- rather than against the bytes the kernel happened to fetch.

    python scripts/roofline_layers.py --batch 1024 --md profiles/pmc/r4_bs1024_roofline.md

Calls mirror the engine's: 1x1 forward with the lazy-BN prologue (x*s+t, ReLU) and the
statistics epilogue, dgrad with the BN-backward fold prologue (g + alpha + beta*y), wgrad with the
fold on g and the lazy-BN transform on x; 3x3 convolutions read operands materialised once
(FDT_MATERIALIZE_3X3: no prologue) and their dgrad runs through the producer's activation.
Minimum bytes per op (1x1 / 3x3):
  fwd   x + W + y            dgrad  g + y + W + dx / g + W + dx + ex     wgrad  g + y + x + dW / g + x + dW
Bound = max(bytes / BW, FLOPs / PEAK) with BW = 6.3 TB/s (the streaming rate measured on this
part, profiles/pmc/calibration.md) and PEAK = 2.5 PFLOP/s dense bf16.
"""
from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch

from bench_conv import SHAPES
from faster_distributed_training_amd.ops import conv_igemm as ci

BW = 6.3e12
PEAK = 2.5e15


def timeit(fn, reps=20):
    """Device time per call: ``reps`` calls captured in one HIP graph and replayed, so small
    launches are not timed at the Python wrapper's host rate (the engine replays graphs too)."""
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(reps):
            fn()
    g.replay()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(3):
        g.replay()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / (3 * reps)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--md", default=None)
    ap.add_argument("--json", default=None)
    ap.add_argument("--keys", default=None,
                    help="engine_launch_keys.py output for this batch: time exactly the (shape, variant) calls "
                         "one engine step makes, weighted by their counts (instead of one variant per shape)")
    a = ap.parse_args()
    dev = torch.device("cuda")
    N = a.batch
    rows = []
    if a.keys:
        return keyed(a, dev)
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
        xb, yb = N * H * H * Cin * 2, M * Cout * 2
        wb = Cout * Cin * k * k * 2
        flops = 2.0 * M * Cout * Cin * k * k
        slab = torch.empty(64 * Cout * shp.ntaps * shp.cxp, device=dev)
        if k > 1:
            # the engine's 3x3 variants: input and gradient materialised once (FDT_MATERIALIZE_3X3),
            # so the conv itself has no prologue; dgrad through the producer's activation
            ex = torch.randn(N, H, H, Cin, device=dev).to(torch.bfloat16) if Cin >= 8 else None
            es = torch.ones(Cin, device=dev)
            et = torch.zeros(Cin, device=dev)
            ops = {"fwd": (lambda: ci.conv_fwd(x, wf, shp), xb + wb + yb)}
            if Cin >= 8:
                ops["dgrad"] = (lambda: ci.conv_dgrad(g, None, None, None, wd, shp, (N, H, H, Cin), epi=ci.EPI_ACTBWD,
                                                      ex=ex, es=es, et=et, act=1), yb + wb + 2 * xb)
            ops["wgrad"] = (lambda: ci.conv_wgrad(g, None, None, None, x, shp, gw, slab=slab), yb + xb + 2 * wb)
        else:
            # 1x1: the lazy-BN prologue on the input, the BN-backward fold on the gradient
            ops = {"fwd": (lambda: ci.conv_fwd(x, wf, shp, sv, tv, 1, 1.0), xb + wb + yb)}
            if Cin >= 8:
                ops["dgrad"] = (lambda: ci.conv_dgrad(g, yy, al, be, wd, shp, (N, H, H, Cin)), 2 * yb + wb + xb)
            ops["wgrad"] = (lambda: ci.conv_wgrad(g, yy, al, be, x, shp, gw, sv, tv, 1, slab=slab),
                            2 * yb + xb + 2 * wb)
        for op, (fn, nbytes) in ops.items():
            t = timeit(fn, a.reps) * 1e3  # us
            bound = max(nbytes / BW, flops / PEAK) * 1e6
            rows.append(dict(shape=f"{H}x{H} {Cin}->{Cout} k{k} s{s}", count=cnt, op=op, us=t, min_mb=nbytes / 1e6,
                             gflop=flops / 1e9, bound_us=bound, pct=100.0 * bound / t,
                             limiter="bytes" if nbytes / BW > flops / PEAK else "mfma"))
            r = rows[-1]
            print(f"{r['shape']:26s} x{cnt} {op:5s} {t:8.1f} us  min {r['min_mb']:8.1f} MB {r['gflop']:7.2f} GF  "
                  f"bound {bound:7.1f} us ({r['limiter']})  {r['pct']:5.1f} %", flush=True)
    tot = sum(r["us"] * r["count"] for r in rows)
    totb = sum(r["bound_us"] * r["count"] for r in rows)
    byop = {}
    for r in rows:
        o = byop.setdefault(r["op"], [0.0, 0.0])
        o[0] += r["us"] * r["count"]
        o[1] += r["bound_us"] * r["count"]
    print(f"network convolutions: {tot / 1e3:.3f} ms measured vs {totb / 1e3:.3f} ms algorithmic bound "
          f"({100 * totb / tot:.1f} %); " + ", ".join(f"{k} {v[0] / 1e3:.3f} / {v[1] / 1e3:.3f} ms" for k, v in byop.items()))
    if a.json:
        with open(a.json, "w") as f:
            json.dump(dict(batch=N, rows=rows), f, indent=1)
    if a.md:
        with open(a.md, "w") as f:
            f.write(f"# Per-layer convolution roofline, batch {N} (scripts/roofline_layers.py)\n\n")
            f.write("Measured: device time of the tuned launch (HIP-graph replay of 20 calls, random data, the engine's prologue / "
                    "epilogue variants).  Algorithmic minimum bytes: every operand read once, every result written "
                    f"once (bf16 activations / packed weights, fp32 dW).  Bound = max(bytes / {BW / 1e12:.1f} TB/s, "
                    f"FLOPs / {PEAK / 1e15:.1f} PFLOP/s).\n\n")
            f.write("| layer | count | op | measured us | min MB | GFLOP | bound us | limiter | % of bound |\n")
            f.write("|---|---:|---|---:|---:|---:|---:|---|---:|\n")
            for r in rows:
                f.write(f"| {r['shape']} | {r['count']} | {r['op']} | {r['us']:.1f} | {r['min_mb']:.1f} | "
                        f"{r['gflop']:.2f} | {r['bound_us']:.1f} | {r['limiter']} | {r['pct']:.1f} |\n")
            f.write(f"\nNetwork convolutions (weighted by layer count): **{tot / 1e3:.3f} ms measured vs "
                    f"{totb / 1e3:.3f} ms algorithmic bound ({100 * totb / tot:.1f} %)**; by op: " +
                    ", ".join(f"{k} {v[0] / 1e3:.3f} / {v[1] / 1e3:.3f} ms ({100 * v[1] / v[0]:.0f} %)"
                              for k, v in byop.items()) + ".\n")


def min_bytes(op_key, N, H, shp):
    Ho, Wo = ci.out_hw(H, H, shp)
    M = N * Ho * Wo
    xb, yb = N * H * H * shp.cin * 2, M * shp.cout * 2
    wb = shp.cout * shp.cin * shp.k * shp.k * 2
    return {"fwd0": xb + wb + yb, "fwd1": xb + wb + yb, "fwd3": 3 * xb + wb + yb,
            "dgrad01": yb + wb + 2 * xb, "dgrad21": 2 * yb + wb + 2 * xb, "dgrad22": 2 * yb + wb + xb,
            "wgrad00": yb + xb + 2 * wb, "wgrad10": 2 * yb + xb + 2 * wb, "wgrad11": 2 * yb + xb + 2 * wb}[op_key]


def keyed(a, dev):
    from retune_graph import variant_call
    rows = []
    for line in open(a.keys):
        parts = line.split()
        if not (len(parts) >= 4 and parts[0].count(":") == 6 and parts[2] in ("hit", "MISS")):
            continue
        key, op_key, cnt = parts[0], parts[1], int(parts[3][1:])
        N, H, Cin, Cout, k, s, p = map(int, key.split(":"))
        if N != a.batch:
            continue
        shp = ci.ConvShape(Cin, Cout, k, s, p)
        fn, keep = variant_call(op_key, N, H, shp, dev)
        if fn is None:
            continue
        Ho, Wo = ci.out_hw(H, H, shp)
        flops = 2.0 * N * Ho * Wo * Cout * Cin * k * k
        nbytes = min_bytes(op_key, N, H, shp)
        t = timeit(fn, a.reps) * 1e3
        bound = max(nbytes / BW, flops / PEAK) * 1e6
        rows.append(dict(shape=f"{H}x{H} {Cin}->{Cout} k{k} s{s}", count=cnt, op=op_key, us=t, min_mb=nbytes / 1e6,
                         gflop=flops / 1e9, bound_us=bound, pct=100.0 * bound / t,
                         limiter="bytes" if nbytes / BW > flops / PEAK else "mfma"))
        r = rows[-1]
        print(f"{r['shape']:26s} x{cnt} {op_key:8s} {t:8.1f} us  bound {bound:7.1f} us ({r['limiter']})  {r['pct']:5.1f} %",
              flush=True)
        del keep
    report(a, rows)


def report(a, rows):
    tot = sum(r["us"] * r["count"] for r in rows)
    totb = sum(r["bound_us"] * r["count"] for r in rows)
    byop = {}
    for r in rows:
        o = byop.setdefault(r["op"].rstrip("0123456789"), [0.0, 0.0])
        o[0] += r["us"] * r["count"]
        o[1] += r["bound_us"] * r["count"]
    print(f"network convolutions: {tot / 1e3:.3f} ms measured vs {totb / 1e3:.3f} ms algorithmic bound "
          f"({100 * totb / tot:.1f} %); " + ", ".join(f"{k} {v[0] / 1e3:.3f} / {v[1] / 1e3:.3f} ms" for k, v in byop.items()))
    if a.json:
        with open(a.json, "w") as f:
            json.dump(dict(batch=a.batch, rows=rows), f, indent=1)
    if a.md:
        with open(a.md, "w") as f:
            f.write(f"# Per-layer convolution roofline, batch {a.batch} (scripts/roofline_layers.py --keys)\n\n")
            f.write("Measured: device time of the tuned launch of exactly the calls one engine training step makes "
                    "(variant = tuned-table op key: fwd{prologue}, dgrad{prologue}{epilogue}, wgrad{fold}{input "
                    "transform}; counts from scripts/engine_launch_keys.py), HIP-graph replay of 20 calls, random "
                    "data.  Algorithmic minimum bytes: every operand read once, every result written once (bf16 "
                    f"activations / packed weights, fp32 dW).  Bound = max(bytes / {BW / 1e12:.1f} TB/s, FLOPs / "
                    f"{PEAK / 1e15:.1f} PFLOP/s).\n\n")
            f.write("| layer | count | variant | measured us | min MB | GFLOP | bound us | limiter | % of bound |\n")
            f.write("|---|---:|---|---:|---:|---:|---:|---|---:|\n")
            for r in rows:
                f.write(f"| {r['shape']} | {r['count']} | {r['op']} | {r['us']:.1f} | {r['min_mb']:.1f} | "
                        f"{r['gflop']:.2f} | {r['bound_us']:.1f} | {r['limiter']} | {r['pct']:.1f} |\n")
            f.write(f"\nNetwork convolutions (weighted by call count): **{tot / 1e3:.3f} ms measured vs "
                    f"{totb / 1e3:.3f} ms algorithmic bound ({100 * totb / tot:.1f} %)**; by op: " +
                    ", ".join(f"{k} {v[0] / 1e3:.3f} / {v[1] / 1e3:.3f} ms ({100 * v[1] / v[0]:.0f} %)"
                              for k, v in byop.items()) + ".\n")


if __name__ == "__main__":
    main()
