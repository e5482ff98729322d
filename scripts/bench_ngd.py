#!/usr/bin/env python3
"""NGD optimizer step time on the real parameter sets (ResNet-50 CIFAR / Transformer 6x512),
random gradients, steady state (update and non-update steps of the schedule separately).

    python scripts/bench_ngd.py [--model resnet50|transformer] [--steps 24]
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="resnet50")
    ap.add_argument("--steps", type=int, default=24)
    a = ap.parse_args()
    from faster_distributed_training_amd.optim.ngd import NGD
    from faster_distributed_training_amd.utils.flat import FlatParams
    dev = torch.device("cuda")
    if a.model == "resnet50":
        from faster_distributed_training_amd.models.resnet import resnet50
        m = resnet50(10)
    else:
        from faster_distributed_training_amd.models.transformer import Transformer
        m = Transformer(4, 30522)
    m = m.to(dev)
    f = FlatParams(m, device=dev)
    o = NGD(f, lr=0.01, momentum=0.9, weight_decay=1e-4)
    g = torch.Generator(device=dev).manual_seed(0)
    times = {True: [], False: []}
    for s in range(a.steps):
        f.grad.normal_(generator=g)
        sts = o._states()
        upd = bool(sts) and sts[0]._updating()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        o.step()
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) * 1e3
        if s >= 2:
            times[upd].append(dt)
    n_axes = len(o._states())
    for k, v in times.items():
        if v:
            v.sort()
            print(f"{a.model}: {'update' if k else 'non-update'} steps: median {v[len(v) // 2]:.2f} ms "
                  f"(min {v[0]:.2f}, n={len(v)}), {n_axes} batched axis states")


if __name__ == "__main__":
    main()
