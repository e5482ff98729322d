#!/usr/bin/env python3
"""Convergence of the Jacobi eigensolver on the REAL NGD matrices: run a few Transformer /
ResNet-50 NGD steps (random gradients), capture every Z handed to ``eigh_many``, then solve the
captured batch with a fixed number of sweeps (tol 0) and with the shipped tolerance: per sweep
count the worst relative eigenvalue error vs fp64 LAPACK, the worst eigen-residual
||Z u - c u|| / ||Z||, and the device time of the launch (graph replay of 10)."""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from faster_distributed_training_amd.ops import eigh as E  # noqa: E402
from roofline_layers import timeit  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="transformer")
    ap.add_argument("--steps", type=int, default=14)
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
    flat = FlatParams(m, device=dev)
    opt = NGD(flat, lr=0.01, momentum=0.9, weight_decay=1e-4, overlap_eigh=False)
    captured = []
    orig = E.eigh_many

    def spy(Zs, *args, **kw):
        captured.append([Z.detach().clone() for Z in Zs])
        return orig(Zs, *args, **kw)
    E.eigh_many = spy
    import faster_distributed_training_amd.optim.ngd as ngdmod
    if hasattr(ngdmod, "eigh_many"):
        ngdmod.eigh_many = spy
    g = torch.Generator(device=dev).manual_seed(0)
    for _ in range(a.steps):
        flat.grad.normal_(generator=g)
        opt.step()
    torch.cuda.synchronize()
    E.eigh_many = orig
    print(f"{a.model}: {len(captured)} eigh_many calls captured", flush=True)
    # the last two update steps (steady state: after the 10-step initialisation schedule)
    for ci, Zs in enumerate(captured[-2:]):
        shapes = [tuple(Z.shape) for Z in Zs]
        refs = [torch.linalg.eigh(Z.double(), UPLO="U") for Z in Zs]
        print(f" call {len(captured) - 2 + ci}: shapes {shapes}", flush=True)
        for sw, tol in [(1, 0.0), (2, 0.0), (3, 0.0), (4, 0.0), (5, 0.0), (6, 0.0), (8, 0.0), (15, 0.0),
                        (E.SWEEPS, E.TOL), (E.SWEEPS, 1e-5), (E.SWEEPS, 1e-4)]:
            out = orig(Zs, sw, tol)
            ev, res = 0.0, 0.0
            for Z, (c, U), (cr, Ur) in zip(Zs, out, refs):
                Zs_ = torch.triu(Z.double()) + torch.triu(Z.double(), 1).transpose(1, 2)
                nz = Zs_.flatten(1).norm(dim=1).clamp_min(1e-30)
                ev = max(ev, ((c.double() - cr).abs().max(1).values / cr.abs().max(1).values.clamp_min(1e-30)).max().item())
                r = (Zs_ @ U.double() - U.double() * c.double().unsqueeze(1)).flatten(1).norm(dim=1) / nz
                res = max(res, r.max().item())
            us = timeit(lambda: orig(Zs, sw, tol), 10) * 1e3
            print(f"   sweeps {sw:2d} tol {tol:.0e}: eig rel err {ev:.2e}  residual {res:.2e}  {us:8.1f} us", flush=True)


if __name__ == "__main__":
    main()
