#!/usr/bin/env python3
"""Jacobi eigensolver cost vs accuracy on the NGD matrices the transformer actually produces.

Captures the Z matrices of one steady-state NGD update (transformer, 32 samples / GPU), then
times ``eigh_many`` for a range of sweep limits / tolerances and reports eigenvalue and
reconstruction errors against the fp64 reference (ops/eigh.py eigh_reference).
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import faster_distributed_training_amd.ops.eigh as Emod  # noqa: E402


def main():
    from faster_distributed_training_amd.train.transformer_trainer import TransformerConfig, TransformerTrainer
    caught = []
    orig = Emod.eigh_many

    def grab(Zs, *a, **k):
        caught.append([Z.detach().clone() for Z in Zs])
        return orig(Zs, *a, **k)
    Emod.eigh_many = grab
    tr = TransformerTrainer(TransformerConfig(batch_size=32, synthetic=True, eval=False, plot=False, ngd=True,
                                              length_buckets=(128, 256), epoch=1))
    it = iter(tr.train_loader)
    tr.model.train()
    for _ in range(22):
        tr.train_step(*next(it))
    torch.cuda.synchronize()
    Emod.eigh_many = orig
    Zs = caught[-1]
    print("matrices:", [(tuple(Z.shape)) for Z in Zs], flush=True)
    ref = [Emod.eigh_reference(Z) for Z in Zs]
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for sweeps, tol in [(15, 1e-6), (15, 1e-5), (15, 1e-4), (10, 1e-6), (8, 1e-6), (6, 1e-6), (5, 1e-6), (4, 1e-6),
                        (3, 1e-6), (2, 1e-6)]:
        for _ in range(2):
            out = orig(Zs, sweeps, tol)
        torch.cuda.synchronize()
        s.record()
        for _ in range(5):
            out = orig(Zs, sweeps, tol)
        e.record()
        torch.cuda.synchronize()
        t = s.elapsed_time(e) / 5
        ew, rec, orth = 0.0, 0.0, 0.0
        for Z, (c, U), (cr, Ur) in zip(Zs, out, ref):
            Zs_ = torch.triu(Z) + torch.triu(Z, 1).transpose(1, 2)
            scale = cr.abs().amax(dim=1, keepdim=True).clamp_min(1e-30)
            ew = max(ew, ((c - cr).abs() / scale).max().item())
            R = U @ torch.diag_embed(c) @ U.transpose(1, 2)
            rec = max(rec, ((R - Zs_).flatten(1).norm(dim=1) / Zs_.flatten(1).norm(dim=1).clamp_min(1e-30)).max().item())
            I = torch.eye(U.shape[-1], device=U.device)
            orth = max(orth, (U.transpose(1, 2) @ U - I).abs().max().item())
        print(f"sweeps {sweeps:2d} tol {tol:.0e}: {t:8.3f} ms   max eigval err (rel to |lambda|max) {ew:.2e}  "
              f"recon {rec:.2e}  orth {orth:.2e}", flush=True)


if __name__ == "__main__":
    main()
