#!/usr/bin/env python3
"""Diagnostic: FSDP(model) NGD, plain vs offload with the device optimizer -- the optimizer's
inputs (gradient, parameters) and output (parameters) compared at every step, per slot."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
os.environ.setdefault("MASTER_PORT", "29642")
import torch  # noqa: E402

from faster_distributed_training_amd.train.transformer_trainer import TransformerConfig, TransformerTrainer  # noqa


def run(arm, steps, opt):
    cfg = TransformerConfig(batch_size=16, synthetic=True, eval=False, plot=False, ngd=opt == "ngd", optimizer=opt,
                            fsdp=True, fsdp_offload=arm != "plain", fsdp_offload_optimizer="device",
                            length_buckets=(128, 256), epoch=1, seed=0, extra={"fsdp_static": False})
    tr = TransformerTrainer(cfg)
    rec = []
    inner = tr.optimizer.step

    def step(*a, **k):
        torch.cuda.synchronize()
        g0, d0 = tr.space.grad.detach().cpu().clone(), tr.space.data.detach().cpu().clone()
        out = inner(*a, **k)
        torch.cuda.synchronize()
        rec.append((g0, d0, tr.space.data.detach().cpu().clone()))
        return out
    tr.optimizer.step = step
    it = iter(tr.train_loader)
    tr.model.train()
    for _ in range(steps):
        tr.train_step(*next(it))
    torch.cuda.synchronize()
    tr.fsdp._quiesce()
    return rec, list(tr.space.slots)


def rel(x, y):
    return ((x - y).norm() / (y.norm() + 1e-30)).item()


for opt, arm in (("ngd", "plain"), ("ngd", "device"), ("madgrad", "device")):
    a, slots = run("plain", 2, opt)
    b, _ = run(arm, 2, opt)
    for i, ((ga, da, pa), (gb, db, pb)) in enumerate(zip(a, b)):
        print(f"{opt} plain vs {arm} step {i}: grad in {rel(gb, ga):.2e}  data in {rel(db, da):.2e}  data out {rel(pb, pa):.2e}  "
              f"update {rel(pb - db, pa - da):.2e}", flush=True)
        rows = []
        for s in slots:
            sl = slice(s.offset, s.offset + s.numel)
            rows.append((rel((pb - db)[sl], (pa - da)[sl]), rel(gb[sl], ga[sl]), s.name, tuple(s.shape)))
        rows.sort(reverse=True)
        print("   worst update slots (upd, grad):", [(n, sh, f"{r:.1e}", f"{q:.1e}") for r, q, n, sh in rows[:5]])
