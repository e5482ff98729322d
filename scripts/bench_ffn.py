#!/usr/bin/env python3
"""FFN (d_model 512, d_ff 1024) forward + backward at transformer-bench token counts: fused
GEMM epilogues (ops/ffn.py) vs the unfused composition, and a tile sweep of the two fused
GEMMs.   python scripts/bench_ffn.py [--tokens 32768]"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from faster_distributed_training_amd.models import transformer as T
from faster_distributed_training_amd.ops import ffn


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
    return s.elapsed_time(e) / reps * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, default=32768)
    a = ap.parse_args()
    dev = torch.device("cuda")
    m = T.PositionalWiseFFN(512, 1024, 0.1).to(dev)
    x = torch.randn(a.tokens, 512, device=dev).to(torch.bfloat16).requires_grad_(True)
    g = torch.randn(a.tokens, 512, device=dev).to(torch.bfloat16)

    def step():
        with torch.autocast("cuda", dtype=torch.bfloat16):
            y = m(x)
        y.backward(g)

    for fused in (False, True):
        ffn.FUSED = fused
        print(f"{'fused' if fused else 'unfused'} fwd+bwd {timeit(step):.1f} us", flush=True)
    ffn.FUSED = True
    w1 = m.w_1.weight.detach().to(torch.bfloat16).contiguous()
    b1 = m.w_1.bias.detach().float().contiguous()
    w2t = m.w_2.weight.detach().to(torch.bfloat16).t().contiguous()
    xa = x.detach()
    aa = torch.empty(a.tokens, 1024, device=dev, dtype=torch.bfloat16)
    hh = torch.empty_like(aa)
    gb = torch.zeros(1024, device=dev)
    lib = timeit(lambda: torch.nn.functional.linear(xa, w1, b1.to(torch.bfloat16)))
    print(f"hipBLASLt x W1^T + b1: {lib:.1f} us")
    for t in [(128, 128, 64, 1), (128, 128, 32, 1), (256, 128, 32, 1), (128, 64, 64, 1), (64, 128, 64, 1),
              (128, 128, 64, 2), (64, 128, 64, 2)]:
        f = timeit(lambda: ffn._gemm(xa, w1, aa, ffn.EPI_GELU_FWD, bias=b1, out2=hh, p=0.1, seed=1, tile=t))
        b = timeit(lambda: ffn._gemm(g, w2t, hh, ffn.EPI_GELU_BWD, a_in=aa, gb=gb, p=0.1, seed=1, tile=t))
        print(f"tile {t}: gelu_fwd {f:.1f} us  gelu_bwd {b:.1f} us", flush=True)


if __name__ == "__main__":
    main()
