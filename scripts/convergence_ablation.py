#!/usr/bin/env python3
"""Ablation of the engine's ResNet-18 / MADGRAD convergence gap.

Same learnable synthetic task, batches and initial weights as scripts/convergence.py; every arm
runs over several seeds (seed = model init + batch order) and reports the held-out cross entropy
and accuracy of its final weights:

  fp32          PyTorch fp32 (the reference numerics)
  torch_bf16    PyTorch under bf16 autocast (bf16 arithmetic alone)
  engine_o      HIP engine, CELU join derivative 1 + o/alpha from the bf16 join OUTPUT (round 5)
  engine_z      HIP engine, derivative exp(z/alpha) from the recomputed fp32 pre-activation (fix)
  engine_torchopt  (a) engine forward/backward (z) + the PyTorch MADGRAD update
  torch_hipopt  (b) PyTorch bf16 forward/backward + the HIP MADGRAD kernel
and (d): every engine arm's final weights are ALSO evaluated through the fp32 PyTorch forward
(``*_evalfp32``), separating training numerics from the engine's eval forward / running stats.

    python scripts/convergence_ablation.py --seeds 5 --out profiles/r6/convergence_ablation.json
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import torch.nn.functional as F

from scripts.convergence import make_task


def evaluate(m, task, amp, fast):
    (_, _), (xte, yte) = task
    fp = m.fast_path
    m.fast_path = fast
    m.eval()
    correct, tloss = 0, 0.0
    with torch.no_grad():
        for i in range(0, xte.shape[0], 256):
            xb = xte[i:i + 256]
            with torch.autocast("cuda", dtype=torch.bfloat16, enabled=amp):
                out = m(xb)
            correct += int((out.float().argmax(1) == yte[i:i + 256]).sum())
            tloss += float(F.cross_entropy(out.float(), yte[i:i + 256], reduction="sum"))
    m.fast_path = fp
    return tloss / xte.shape[0], correct / xte.shape[0]


def run(arm, task, seed, steps, bs, arch="resnet18", lr=2e-3):
    from faster_distributed_training_amd.models import resnet as R
    from faster_distributed_training_amd.ops import resnet_fused as RF
    from faster_distributed_training_amd.optim import flat_optim as O
    from faster_distributed_training_amd.utils.flat import FlatParams
    engine = arm.startswith("engine")
    amp = arm != "fp32"
    os.environ["FDT_NATIVE"] = "1" if engine else "0"
    RF.CELU_ZGRAD = arm != "engine_o"
    (xtr, ytr), _ = task
    torch.manual_seed(seed)
    m = getattr(R, arch)(10).cuda()
    m.fast_path = engine
    flat = FlatParams(m, device="cuda")
    o = O.MADGRAD(flat, lr=lr, momentum=0.9, weight_decay=5e-4)
    if arm == "engine_torchopt":
        o._native = False
    if arm == "torch_hipopt":
        o._native = True
    clip = O.GradClipper(flat)
    g = torch.Generator(device="cpu").manual_seed(seed + 1)
    m.train()
    t0 = time.perf_counter()
    for _ in range(steps):
        idx = torch.randint(0, xtr.shape[0], (bs,), generator=g).cuda()
        x, y = xtr[idx], ytr[idx]
        with torch.autocast("cuda", dtype=torch.bfloat16, enabled=amp):
            out = m(x)
        loss = F.cross_entropy(out.float(), y)
        loss.backward()
        clip(10.0)
        o.step(grad_scale=clip.coef)
    torch.cuda.synchronize()
    res = {"seconds": time.perf_counter() - t0}
    res["test_loss"], res["test_acc"] = evaluate(m, task, amp, engine)
    if engine:
        os.environ["FDT_NATIVE"] = "0"
        res["evalfp32_loss"], res["evalfp32_acc"] = evaluate(m, task, False, False)
    os.environ["FDT_NATIVE"] = "1"
    RF.CELU_ZGRAD = True
    return res


ARMS = ["fp32", "torch_bf16", "engine_o", "engine_z", "engine_torchopt", "torch_hipopt"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seeds", type=int, default=5)
    ap.add_argument("--steps", type=int, default=300)
    ap.add_argument("--bs", type=int, default=128)
    ap.add_argument("--arms", default=",".join(ARMS))
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    task = make_task(device="cuda")
    arms = a.arms.split(",")
    res = {arm: [] for arm in arms}
    for seed in range(a.seeds):
        for arm in arms:
            r = run(arm, task, seed, a.steps, a.bs)
            res[arm].append(r)
            print(f"seed {seed} {arm:16s} held-out CE {r['test_loss']:.4f} acc {r['test_acc']:.3f}"
                  + (f"  | fp32-eval CE {r['evalfp32_loss']:.4f} acc {r['evalfp32_acc']:.3f}"
                     if "evalfp32_loss" in r else "") + f"  ({r['seconds']:.1f} s)", flush=True)
    print("\nsummary (median over seeds; [min, max]):")
    summ = {}
    for arm, rs in res.items():
        for key in ("test_loss", "test_acc", "evalfp32_loss", "evalfp32_acc"):
            vals = [r[key] for r in rs if key in r]
            if not vals:
                continue
            summ[f"{arm}.{key}"] = {"median": statistics.median(vals), "min": min(vals), "max": max(vals),
                                    "values": vals}
            print(f"  {arm:16s} {key:14s} {statistics.median(vals):.4f}  [{min(vals):.4f}, {max(vals):.4f}]")
    if a.out:
        os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
        with open(a.out, "w") as f:
            json.dump({"args": vars(a), "runs": res, "summary": summ}, f, indent=1)


if __name__ == "__main__":
    main()
