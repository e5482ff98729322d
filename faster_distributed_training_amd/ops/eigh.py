"""Batched symmetric eigendecomposition for the NGD preconditioner (K13 / A7).

NGD needs ``eigh`` of many small (rank <= 80) symmetric matrices per update step
(reference ``ngd_optimizer.py:265`` calls LAPACK/cuSOLVER once per (parameter, axis)).
On MI355X all matrices of a step go through ``csrc/kernels/eigh.hip``: one workgroup per
matrix, the matrix and its eigenvector accumulator resident in LDS (2 x 80 x 80 fp32 =
51 KB), cyclic two-sided Jacobi with round-robin parallel ordering (n/2 disjoint
rotations per round, one wave64-wide pass per rotation set), sorted ascending.
"""
from __future__ import annotations

import torch

from . import _native


def eigh_reference(Z: torch.Tensor):
    """(eigenvalues ascending [G,n], eigenvectors [G,n,n] as columns) in fp64 math."""
    c, U = torch.linalg.eigh(Z.double(), UPLO="U")
    return c.to(Z.dtype), U.to(Z.dtype)


def batched_eigh(Z: torch.Tensor, sweeps: int = 12):
    if Z.is_cuda and _native.enabled():
        nat = _native.native()
        if hasattr(nat, "jacobi_eigh") and Z.shape[-1] <= 128 and Z.dtype == torch.float32:
            G, n, _ = Z.shape
            A = Z.contiguous()
            w = torch.empty(G, n, device=Z.device, dtype=torch.float32)
            V = torch.empty(G, n, n, device=Z.device, dtype=torch.float32)
            nat.jacobi_eigh(A.data_ptr(), w.data_ptr(), V.data_ptr(), G, n, sweeps, _native.stream_ptr())
            return w, V
        return torch.linalg.eigh(Z)
    return eigh_reference(Z)
