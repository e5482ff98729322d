"""Batched symmetric eigendecomposition for the NGD preconditioner (K13 / A7).

NGD needs ``eigh`` of many small (rank <= 80) symmetric matrices per update step
(reference ``ngd_optimizer.py:265`` calls LAPACK/cuSOLVER once per (parameter, axis)).
On MI355X the matrices go through ``csrc/kernels/eigh.hip``: one workgroup per matrix, the
matrix and its eigenvector accumulator resident in LDS (2 x 80 x 81 fp32 = 52 KB), cyclic
two-sided Jacobi with round-robin parallel ordering (n/2 disjoint rotations per round),
sorted ascending.  ``eigh_many`` takes matrices of DIFFERENT sizes (every NGD shape group
of one axis level) and runs them in ONE launch through the kernel's ragged table.
"""
from __future__ import annotations

import os

import torch

from . import _native

MAX_N = 128
SWEEPS = 15
TOL = 1e-6
# the NGD preconditioner's solves stop at off-diagonal mass <= 1e-5 ||Z||_F: on the real NGD
# matrices (scripts/eigh_probe.py, profiles/r5/eigh_probe_*.txt) the eigenvalues are at the fp32
# floor (1.4-2.2e-6 relative) from sweep 5 on, the eigen-residual is ~1e-5 (1e-6 at TOL), and
# every sweep costs ~100 us of the update step's critical path: 6-7 sweeps instead of 8
# (the reference only asserts W W^T ~ diag within 0.1, ngd_optimizer.py:343-345)
NGD_TOL = float(os.environ.get("FDT_NGD_EIGH_TOL", "1e-5"))


def eigh_reference(Z: torch.Tensor):
    """(eigenvalues ascending [G,n], eigenvectors [G,n,n] as columns) in fp64 math."""
    c, U = torch.linalg.eigh(Z.double(), UPLO="U")
    return c.to(Z.dtype), U.to(Z.dtype)


def _use_native(Z):
    return Z.is_cuda and _native.enabled() and Z.shape[-1] <= MAX_N and Z.dtype == torch.float32


def batched_eigh(Z: torch.Tensor, sweeps: int = SWEEPS, tol: float = TOL):
    """Ascending eigenvalues [G,n] and eigenvector columns [G,n,n] of symmetric Z [G,n,n]
    (upper triangle read).  GPU: one HIP workgroup per matrix (no host round trip)."""
    if _use_native(Z):
        nat = _native.native()
        G, n, _ = Z.shape
        A = Z.contiguous()
        w = torch.empty(G, n, device=Z.device, dtype=torch.float32)
        V = torch.empty(G, n, n, device=Z.device, dtype=torch.float32)
        nat.jacobi_eigh(A.data_ptr(), w.data_ptr(), V.data_ptr(), 0, G, n, sweeps, tol, _native.stream_ptr())
        return w, V
    # everything else: fp64, upper triangle -- the reference's CPU eigh (ngd_optimizer.py:262-265).
    # (fp32 rocSOLVER on the lower triangle, the previous GPU fallback, read a slightly
    # different Z -- L = J W^T is not symmetric -- and lost the near-degenerate eigenvectors of
    # the initialisation schedule: the FDT_NATIVE=0 NGD run diverged within 20 steps,
    # profiles/r4/convergence_first_run_ngd_lr0.05.json)
    return eigh_reference(Z)


_TABLES: dict = {}


def _table(shapes, device):
    """Device table [(n, offA, offw)] per matrix (cached: NGD shapes repeat every step),
    largest matrices first so the long-running workgroups start earliest."""
    key = (tuple(shapes), str(device))
    hit = _TABLES.get(key)
    if hit is None:
        rows, offA, offw, slices = [], 0, 0, []
        for G, n in shapes:
            slices.append((offA, offw))
            for g in range(G):
                rows.append((n, offA + g * n * n, offw + g * n))
            offA += G * n * n
            offw += G * n
        rows.sort(key=lambda r: -r[0])
        tab = torch.tensor(rows, dtype=torch.int32).view(-1).to(device)
        hit = (tab, len(rows), offA, offw, slices)
        _TABLES[key] = hit
    return hit


def eigh_many(Zs, sweeps: int = SWEEPS, tol: float = TOL):
    """``[batched_eigh(Z) for Z in Zs]`` for symmetric Z_i [G_i, n_i, n_i] of mixed sizes —
    one kernel launch on the native path."""
    if not Zs:
        return []
    if len(Zs) == 1 or not all(_use_native(Z) for Z in Zs):
        return [batched_eigh(Z, sweeps, tol) for Z in Zs]
    nat = _native.native()
    dev = Zs[0].device
    shapes = [(Z.shape[0], Z.shape[-1]) for Z in Zs]
    tab, nmat, totA, totw, slices = _table(shapes, dev)
    A = torch.cat([Z.reshape(-1) for Z in Zs])
    w = torch.empty(totw, device=dev, dtype=torch.float32)
    V = torch.empty(totA, device=dev, dtype=torch.float32)
    nmax = max(n for _, n in shapes)
    nat.jacobi_eigh(A.data_ptr(), w.data_ptr(), V.data_ptr(), tab.data_ptr(), nmat, nmax, sweeps, tol,
                    _native.stream_ptr())
    out = []
    for (G, n), (oa, ow) in zip(shapes, slices):
        out.append((w[ow:ow + G * n].view(G, n), V[oa:oa + G * n * n].view(G, n, n)))
    return out
