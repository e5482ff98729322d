#!/usr/bin/env python3
"""dst(fp32) += dY^T X for the transformer's linear layers at the 8-GPU per-GPU share (32
samples: 4096-8192 tokens) and at 256 samples: the split-K batched GEMM + slab fold the
engine uses (ops/linear.py wgrad_into: two launches) against one library GEMM accumulating
into the fp32 gradient (addmm, out_dtype fp32, beta 1).  Device time per call from a
captured HIP graph of 20 calls.

    python scripts/bench_wgrad_accum.py
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def gtime(fn, reps=20):
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
    return s.elapsed_time(e) / (3 * reps) * 1e3


def main():
    from faster_distributed_training_amd.ops.linear import wgrad_into
    dev = torch.device("cuda")
    tot = {}
    for M in (4096, 8192, 32768):
        for fin, fout in [(512, 1536), (512, 512), (512, 2048), (2048, 512)]:
            torch.manual_seed(0)
            x = torch.randn(M, fin, device=dev).to(torch.bfloat16)
            g = torch.randn(M, fout, device=dev).to(torch.bfloat16)
            ref = g.double().t() @ x.double()
            d1 = torch.zeros(fout, fin, device=dev)
            d2 = torch.zeros(fout, fin, device=dev)
            t1 = gtime(lambda: wgrad_into(g, x, d1))
            try:
                t2 = gtime(lambda: torch.addmm(d2, g.t(), x, out_dtype=torch.float32, out=d2))
                d2.zero_()
                torch.addmm(d2, g.t(), x, out_dtype=torch.float32, out=d2)
                e2 = ((d2.double() - ref).norm() / ref.norm()).item()
            except Exception as ex:  # noqa: BLE001
                t2, e2 = float("nan"), repr(ex)[:80]
            d1.zero_()
            wgrad_into(g, x, d1)
            e1 = ((d1.double() - ref).norm() / ref.norm()).item()
            tot.setdefault(M, [0.0, 0.0])
            tot[M][0] += t1
            tot[M][1] += t2
            print(f"M {M:6d} {fin:5d}->{fout:5d}: split-K + fold {t1:7.1f} us (err {e1:.1e})   addmm beta=1 {t2:7.1f} us "
                  f"(err {e2 if isinstance(e2, str) else f'{e2:.1e}'})", flush=True)
    for M, (a, b) in tot.items():
        print(f"M {M}: totals split-K {a:.1f} us, addmm {b:.1f} us", flush=True)


if __name__ == "__main__":
    main()
