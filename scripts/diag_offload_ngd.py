#!/usr/bin/env python3
"""Diagnostic: per-slot update differences of FSDP(model) NGD, plain vs offload-device optimizer."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
os.environ.setdefault("MASTER_PORT", "29642")
import torch  # noqa: E402

from faster_distributed_training_amd.train.transformer_trainer import TransformerConfig, TransformerTrainer  # noqa


def run(arm, steps):
    cfg = TransformerConfig(batch_size=16, synthetic=True, eval=False, plot=False, ngd=True, optimizer="ngd", fsdp=True,
                            fsdp_offload=arm != "plain", fsdp_offload_optimizer="device", length_buckets=(128, 256),
                            epoch=1, seed=0, extra={"fsdp_static": False})
    tr = TransformerTrainer(cfg)
    fs = tr.fsdp
    it = iter(tr.train_loader)
    tr.model.train()
    fs._quiesce()
    init = fs.shard_data.clone().cpu()
    g = []
    for _ in range(steps):
        tr.train_step(*next(it))
        torch.cuda.synchronize()
        fs._quiesce()
        g.append(tr.space.grad.detach().cpu().clone())
    upd = fs.shard_data.cpu() - init
    return upd, g, [s for s in tr.space.slots], tr.optimizer


for steps in (1, 2, 3):
    a, ga, slots, oa = run("plain", steps)
    b, gb, _, ob = run("device", steps)
    print(f"steps {steps}: update rel diff {((a - b).norm() / a.norm()).item():.3e}; grad rel diff per step",
          [f"{((x - y).norm() / (x.norm() + 1e-30)).item():.2e}" for x, y in zip(ga, gb)])
    rows = []
    for s in slots:
        da, db = a[s.offset:s.offset + s.numel], b[s.offset:s.offset + s.numel]
        rows.append((((da - db).norm() / (da.norm() + 1e-30)).item(), s.name, s.numel))
    rows.sort(reverse=True)
    print("   worst slots:", [(n, f"{r:.2e}") for r, n, _ in rows[:6]])
    print("   opt state keys plain:", sorted(getattr(oa, "state", {}).get("__flat__", {}).keys())[:8])
