#!/usr/bin/env python3
"""Linear-layer weight gradient dW = dY^T X (tokens x features, bf16) on MI355X: the library
GEMM PyTorch's autograd issues, a split-K batched GEMM, and the MFMA wgrad kernel of the
conv engine (1x1 "direct" mode: split-K with fp32 atomics straight into the fp32 gradient).

    python scripts/bench_linear_wgrad.py [--tokens 32768]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters * 1e3  # us


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, default=32768)
    a = ap.parse_args()
    from faster_distributed_training_amd.ops import conv_igemm as ci
    dev = torch.device("cuda")
    M = a.tokens
    for fin, fout in [(512, 1536), (512, 512), (512, 1024), (1024, 512)]:
        x = torch.randn(M, fin, device=dev).to(torch.bfloat16)
        g = torch.randn(M, fout, device=dev).to(torch.bfloat16)
        ref = g.float().t() @ x.float()
        t_lib = timeit(lambda: g.t() @ x)

        def splitk(s=8, f32=False):
            if f32:
                p = torch.bmm(g.view(s, M // s, fout).transpose(1, 2), x.view(s, M // s, fin), out_dtype=torch.float32)
                return p.sum(0)
            p = torch.bmm(g.view(s, M // s, fout).transpose(1, 2), x.view(s, M // s, fin))
            return p.float().sum(0)
        sk = {}
        for s in (4, 8, 16, 32):
            sk[s] = timeit(lambda: splitk(s))
        try:
            e32 = ((splitk(8, True) - ref).norm() / ref.norm()).item()
            sk["f32out8"] = timeit(lambda: splitk(8, True))
            sk["f32out16"] = timeit(lambda: splitk(16, True))
            sk["f32err"] = e32
        except Exception as e:  # noqa: BLE001
            sk["f32out"] = repr(e)[:60]
        sk["bf16err"] = ((splitk(8) - ref).norm() / ref.norm()).item()
        print("  split-K:", {k: (round(v, 1) if isinstance(v, float) and v > 1e-3 else v) for k, v in sk.items()})
        t_sk = sk[8]
        out = torch.empty(fout, fin, device=dev)
        shp = ci.ConvShape(fin, fout, 1, 1, 0)
        fn = lambda: ci.conv_wgrad(g.view(M, 1, 1, fout), None, None, None, x.view(M, 1, 1, fin), shp, out)
        t_wg = timeit(fn)
        fn()
        torch.cuda.synchronize()
        err = ((out - ref).norm() / ref.norm()).item()
        from faster_distributed_training_amd.ops.linear import bias_grad
        t_bsum = timeit(lambda: g.sum(0, dtype=torch.float32))
        t_bgemv = timeit(lambda: bias_grad(g))
        print(f"  bias grad: column sum {t_bsum:.1f} us, GEMV {t_bgemv:.1f} us "
              f"(rel diff {((bias_grad(g) - g.float().sum(0)).norm() / g.float().sum(0).norm()).item():.1e})")
        gf = 2.0 * M * fin * fout / 1e9
        print(f"in {fin:5d} out {fout:5d}: library {t_lib:7.1f} us ({gf / t_lib:6.1f} TF/s)  split-K bmm {t_sk:7.1f} us  "
              f"MFMA wgrad {t_wg:7.1f} us ({gf / t_wg:6.1f} TF/s, rel err {err:.1e})", flush=True)


if __name__ == "__main__":
    main()
