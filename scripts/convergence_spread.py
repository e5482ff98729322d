#!/usr/bin/env python3
"""Run-to-run spread of the convergence task's held-out statistics (scripts/convergence.py): the
ResNet engine arm N times (non-deterministic fp32 atomics), once in deterministic mode, the fp32
PyTorch arm M times -- is an engine outlier (held-out loss far above its twins) engine-specific?"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from convergence import make_task, train_curve  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--arch", default="resnet50")
    ap.add_argument("--opt", default="madgrad")
    ap.add_argument("--engine", type=int, default=8)
    ap.add_argument("--ref", type=int, default=3)
    ap.add_argument("--steps", type=int, default=300)
    a = ap.parse_args()
    task = make_task(device="cuda")
    kw = dict(device="cuda", task=task, arch=a.arch, bs=128)
    for i in range(a.engine):
        r = train_curve(True, a.opt, a.steps, **kw)
        print(f"engine   {i}: held-out loss {r['test_loss']:.4f} acc {r['test_acc']:.4f}", flush=True)
    from faster_distributed_training_amd.ops import _native
    _native.set_deterministic(True)
    r = train_curve(True, a.opt, a.steps, **kw)
    _native.set_deterministic(False)
    print(f"engine det : held-out loss {r['test_loss']:.4f} acc {r['test_acc']:.4f}", flush=True)
    for i in range(a.ref):
        r = train_curve(False, a.opt, a.steps, bf16=False, **kw)
        print(f"fp32     {i}: held-out loss {r['test_loss']:.4f} acc {r['test_acc']:.4f}", flush=True)


if __name__ == "__main__":
    main()
