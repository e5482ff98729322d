#!/usr/bin/env python3
"""Host-side profile (cProfile) of steady-state training steps: where the Python time of a
host-bound step goes (transformer at 32 samples / GPU: host ~4.2 of 4.9 ms per step).

    python scripts/host_profile.py --model transformer --batch 32 --steps 50
"""
import argparse
import cProfile
import io
import os
import pstats
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="transformer", choices=["transformer", "resnet50"])
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--top", type=int, default=30)
    a = ap.parse_args()
    if a.model == "transformer":
        from faster_distributed_training_amd.train.transformer_trainer import TransformerConfig, TransformerTrainer
        tr = TransformerTrainer(TransformerConfig(batch_size=a.batch, synthetic=True, eval=False, plot=False, ngd=True,
                                                  length_buckets=(128, 256), epoch=1))
        it = iter(tr.train_loader)
        step = lambda: tr.train_step(*next(it))  # noqa: E731
    else:
        from faster_distributed_training_amd.train.resnet_trainer import ResNetConfig, ResNetTrainer
        tr = ResNetTrainer(ResNetConfig(arch="resnet50", bs=a.batch, synthetic=True, eval=False, plot=False))

        def gen():
            while True:
                for b in tr.train_loader:
                    yield b
        it = gen()
        step = lambda: tr.train_step(*next(it))  # noqa: E731
    tr.model.train()
    for _ in range(15):
        step()
    torch.cuda.synchronize()
    pr = cProfile.Profile()
    t0 = time.perf_counter()
    pr.enable()
    for _ in range(a.steps):
        step()
    pr.disable()
    host = (time.perf_counter() - t0) / a.steps * 1e3
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / a.steps * 1e3
    print(f"{a.model} batch {a.batch}: host {host:.3f} ms / step under cProfile, wall {wall:.3f} ms / step")
    for key in ("tottime", "cumulative"):
        s = io.StringIO()
        pstats.Stats(pr, stream=s).sort_stats(key).print_stats(a.top)
        print(f"---- by {key} ----")
        print("\n".join(s.getvalue().splitlines()[:a.top + 12]))


if __name__ == "__main__":
    main()
