#!/usr/bin/env python3
"""Diagnostic for test_sharded_ngd_graphs_world2: the unsharded and sharded NGD runs (two gloo
ranks on one GPU, deterministic engine) step by step -- max |difference| of every parameter
after each step, so the first step at which the two runs part (and how fast) is visible.

    python scripts/diag_sharded_h3.py
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
from dist_utils import run_world  # noqa: E402

STEPS = 16


def worker(rank, world):
    import torch
    from faster_distributed_training_amd.train.resnet_trainer import ResNetConfig, ResNetTrainer
    torch.cuda.set_device(0)
    base = dict(arch="resnet18", bs=16, synthetic=True, eval=False, plot=False, ngd=True, optimizer="ngd",
                distributed=True, deterministic=True, extra={"subset_stride": 50},
                clip=float(os.environ.get("CLIP", "10")))
    arms = [a == "1" for a in os.environ.get("ARMS", "0,1").split(",")]
    hist = {}
    for ai, shard in enumerate(arms):
        tr = ResNetTrainer(ResNetConfig(shard_ngd=shard, bucket_mb=2.0, first_bucket_mb=0.5, **base))
        it = iter(tr.train_loader)
        h = []
        for _ in range(STEPS):
            x, y = next(it)
            tr.train_step(x, y)
            torch.cuda.synchronize()
            h.append(({k: v.detach().float().clone() for k, v in tr.model.state_dict().items()
                       if v.dtype.is_floating_point}, tr.clipper.norm.item()))
        hist[ai] = h
    if rank == 0:
        for p, q in zip(range(0, len(arms), 2), range(1, len(arms), 2)):
            print(f"arms {p} (shard={arms[p]}) vs {q} (shard={arms[q]})", flush=True)
            for i, ((a, xa), (b, xb)) in enumerate(zip(hist[p], hist[q])):
                worst = max(((b[k] - a[k]).abs().max().item(), k) for k in a)
                print(f"step {i}: grad norms {xa:.9e} / {xb:.9e}; max |diff| {worst[0]:.3e} ({worst[1]})", flush=True)


if __name__ == "__main__":
    run_world(worker, world=2, native=True, timeout=600)
