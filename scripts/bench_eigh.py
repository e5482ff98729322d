#!/usr/bin/env python3
"""Jacobi eigh launch time on NGD-like matrices (low rank + ridge), G matrices of size n."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch


def main():
    from faster_distributed_training_amd.ops.eigh import batched_eigh
    dev = torch.device("cuda")
    for G, n in [(16, 80), (58, 80), (16, 32)]:
        torch.manual_seed(0)
        B = torch.randn(G, n, n // 2, device=dev)
        Z = B @ B.transpose(1, 2) / n + 1e-3 * torch.eye(n, device=dev)
        for _ in range(3):
            batched_eigh(Z)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(10):
            batched_eigh(Z)
        torch.cuda.synchronize()
        print(f"eigh G={G} n={n}: {(time.perf_counter() - t0) / 10 * 1e3:.3f} ms")


if __name__ == "__main__":
    main()
