"""Online natural-gradient descent (NG-SGD, Povey et al.) — batched, sync-free.

Reference: ``ngd_optimizer.py`` — ``OnlineNaturalGradient`` (``:8-420``: a low-rank-plus-
identity inverse-Fisher factor per tensor axis) and ``NGD`` (``:423-508``: weight decay ->
per-axis preconditioning -> SGD momentum).  Same mathematics, re-designed for MI355X:

* **batched**: all parameters with the same shape are stacked; each axis of a shape
  group is one set of batched GEMMs (``[G,N,D] x [G,D,R]``) instead of one Python object
  per (parameter, axis) — ResNet-50's 157 live preconditioners collapse into a few
  dozen groups;
* **no host synchronisation**: every scalar the reference pulls to the host with
  ``.item()`` (~943 per step measured, survey A7) — trace(K), rho, tr(D), floors, the
  NaN guard — stays a device tensor; the update schedule depends only on the host step
  counter;
* **eigendecomposition**: each preconditioner is written as a generator that yields its
  rank x rank (<= 80) symmetric Z matrix and resumes with the eigenpairs; the optimizer
  drives all shape groups in lock-step, so every Z of one axis level goes through ONE
  ragged launch (``ops/eigh.py::eigh_many``: the HIP one-workgroup-per-matrix Jacobi
  kernel on MI355X) instead of one solver call per (parameter, axis);
* the final momentum/weight update is the fused flat SGD kernel (``optim/flat_optim.py``).
"""
from __future__ import annotations

import math
import os

import torch

from ..ops import _native
from ..utils.flat import FlatParams
from .flat_optim import SGD

EPSILON = 1.0e-10
DELTA = 5.0e-4


def default_rank(dim: int, rank: int = -1) -> int:
    if rank >= 0:
        assert 0 < rank < dim
        return rank
    return min((dim + 1) // 2, 80)


def orthonormal_special(rank: int, dim: int, dtype=torch.float32, device=None) -> torch.Tensor:
    """Deterministic near-orthonormal [rank, dim] initial factor (``ngd_optimizer.py:397-420``):
    a scaled identity block (first element 1.1) followed by repeated identity blocks,
    rows normalised."""
    first = 1.1
    ncols = dim // rank
    rem = dim % rank
    k = torch.full((rank,), 1.0 / math.sqrt(first * first + ncols - 1), dtype=dtype, device=device)
    k[:rem] = 1.0 / math.sqrt(first * first + ncols)
    eye = torch.diag(k)
    blocks = [torch.diag(k * first)] + [eye] * (ncols + 1)
    return torch.cat(blocks, dim=1)[:, :dim].contiguous()


FUSED = os.environ.get("FDT_NGD_FUSED", "1") != "0"
# one eigensolver launch per optimizer step for all update-step Z matrices (see Deferred)
DEFER = os.environ.get("FDT_NGD_DEFER", "1") != "0"
# steady-state optimizer steps replayed as HIP graphs (NGD._graph_step).  Off by default:
# measured on MI355X (profiles/r3/ngd_graphs.txt) a replay is no faster than the eager step
# (ResNet-50 NGD+meta 30.4 vs 30.2-30.7 ms, transformer bs256 11.5 vs 11.4-12.2 ms) and slower
# at batch 32 (5.39 vs 5.04 ms): the step is GPU-bound, not launch-bound.  FDT_NGD_GRAPHS=1
# forces it on everywhere; the ResNet trainer turns it on for the sharded path, where a rank
# preconditions 1/world of the parameters and the step IS launch-bound (train/resnet_trainer.py)
GRAPHS = os.environ.get("FDT_NGD_GRAPHS", "0") == "1"
# plain (non-update) steps without weight decay: the clip coefficient applied by the SGD kernel
# instead of a pass over the flat gradient (NGD._scale_deferrable)
DEFER_SCALE = os.environ.get("FDT_NGD_DEFER_SCALE", "1") != "0"
# the R x R products of an update step (K = J J^T, L = J W^T, W <- A (J + wc W)) on the
# hand-written ngd.hip kernels (ngd_gram / ngd_wupdate) instead of batched library GEMMs
SMALL_GEMM = os.environ.get("FDT_NGD_GEMM", "1") != "0"


def _gemm_native(J) -> bool:
    return SMALL_GEMM and J.is_cuda and _native.enabled() and hasattr(_native.native(), "ngd_gram")


def gram(J, W=None):
    """(K = J J^T, L = J W^T or None) for J, W [G, R, D] fp32 -- ngd_gram (split-d partial tiles
    summed in a fixed order) or two batched GEMMs."""
    if not _gemm_native(J):
        K = torch.bmm(J, J.transpose(1, 2))
        return K, (torch.bmm(J, W.transpose(1, 2)) if W is not None else None)
    nat = _native.native()
    G, R, D = J.shape
    Jc = J.contiguous()
    Wc = W.contiguous() if W is not None else None
    K = torch.empty(G, R, R, device=J.device, dtype=torch.float32)
    L = torch.empty(G, R, R, device=J.device, dtype=torch.float32) if W is not None else None
    slab = torch.empty(nat.ngd_gram_slab_numel(G, R, D, W is not None), device=J.device, dtype=torch.float32)
    nat.ngd_gram(Jc.data_ptr(), Wc.data_ptr() if Wc is not None else 0, K.data_ptr(),
                 L.data_ptr() if L is not None else 0, slab.data_ptr(), G, R, D, _native.stream_ptr())
    return K, L


def w_update(A, J, wc, W):
    """W <- A (J + wc W) in place (W, J [G, R, D]; A [G, R, R]; wc [G, R])."""
    if not (_gemm_native(J) and W.is_contiguous()):
        torch.bmm(A, torch.addcmul(J, wc.unsqueeze(2), W), out=W)
        return
    G, R, D = W.shape
    Ac, Jc, wcc = A.contiguous(), J.contiguous(), wc.contiguous()
    _native.native().ngd_wupdate(Ac.data_ptr(), Jc.data_ptr(), wcc.data_ptr(), W.data_ptr(), G, R, D,
                                 _native.stream_ptr())


def _fused_small_math(X, R) -> bool:
    return (FUSED and X.is_cuda and X.dtype == torch.float32 and R <= 128 and _native.enabled()
            and hasattr(_native.native(), "ngd_pre_eigh"))


def _native_eigh(device) -> bool:
    """Capturable only with the HIP Jacobi eigh (hipSOLVER's syevd is not graph-safe)."""
    from ..ops import eigh as E
    return E._use_native(torch.empty(1, 2, 2, device=device))


class Deferred:
    """A Z matrix whose eigenpairs only feed the preconditioner's NEXT step (the W / d / rho
    update): the generator goes on without waiting, and ``drive`` solves every deferred Z of
    the whole optimizer step in one eigensolver launch at the end, then calls ``fn(c, U)``."""
    __slots__ = ("Z", "fn")

    def __init__(self, Z, fn):
        self.Z, self.fn = Z, fn


def drive(gens, side=None, defer_out=None):
    """Run preconditioner generators in lock-step: each yields a batch of Z matrices and
    receives ``(eigenvalues, eigenvectors)``; all Z pending at the same time are solved by
    one ``eigh_many`` launch.  ``Deferred`` yields are collected and solved together after
    all generators finished (one launch for all axes instead of one per axis level).
    Returns the generators' return values.

    ``side`` (a HIP stream): the deferred solve and the state updates it feeds run there,
    concurrently with whatever the caller's stream does next (the next training step): the
    eigensolver occupies one workgroup per matrix -- 16-60 of the 256 CUs -- for ~1 ms, and
    its results are only read by the next optimizer step.  ``drive`` then also returns
    ``(done_event, keepalive)``: the caller's stream must wait on the event before the state
    is read again, and ``keepalive`` (the deferred inputs, made on the caller's stream) must
    outlive that wait.

    ``defer_out`` (a list): the deferred work is appended to it instead of being solved (the
    HIP-graph path captures it as a separate graph on the side stream)."""
    from ..ops.eigh import NGD_TOL, eigh_many
    results = [None] * len(gens)
    deferred = []

    def advance(i, val, first=False):
        g = gens[i]
        try:
            out = next(g) if first else g.send(val)
            while isinstance(out, Deferred):
                deferred.append(out)
                out = g.send(None)
            return out
        except StopIteration as e:
            results[i] = e.value
            return None

    pending = {}
    for i in range(len(gens)):
        z = advance(i, None, first=True)
        if z is not None:
            pending[i] = z
    while pending:
        idx = list(pending)
        outs = eigh_many([pending[i] for i in idx], tol=NGD_TOL)
        pending = {}
        for i, o in zip(idx, outs):
            z = advance(i, o)
            if z is not None:
                pending[i] = z
    if defer_out is not None:
        defer_out.extend(deferred)
        return results
    if side is not None:
        if not deferred:
            return results, None
        side.wait_stream(torch.cuda.current_stream(side.device))
        with torch.cuda.stream(side):
            for d, (c, U) in zip(deferred, eigh_many([d.Z for d in deferred], tol=NGD_TOL)):
                d.fn(c, U)
            done = torch.cuda.Event()
            done.record(side)
        return results, (done, deferred)
    if deferred:
        for d, (c, U) in zip(deferred, eigh_many([d.Z for d in deferred], tol=NGD_TOL)):
            d.fn(c, U)
    return results


class NGState:
    """Batched state of G preconditioners sharing (dim, rank)."""

    def __init__(self, G, dim, rank, alpha, update_period, eta, dtype, device):
        self.G, self.dim, self.rank = G, dim, rank
        self.alpha, self.update_period, self.eta = float(alpha), int(update_period), float(eta)
        self.t = 0
        self.dtype, self.device = dtype, device
        self.W = None
        self.d = None
        self.rho = None
        self.last_ip = None  # per-matrix |X|^2 of the last call (HIP path), handed to the next axis
        # HIP path: defer the eigensolve of an update to the end of the optimizer step (off
        # only inside the initialisation iterations, where each one needs the previous W)
        self.defer = True

    # -------------------------------------------------------------- schedule
    def _updating(self):
        return self.t < 10 or self.t % self.update_period == 0

    def _init_default(self):
        R, D = self.rank, self.dim
        self.rho = torch.full((self.G,), EPSILON, dtype=self.dtype, device=self.device)
        self.d = torch.full((self.G, R), EPSILON, dtype=self.dtype, device=self.device)
        e_tii = 1.0 / (2.0 + (D + R) * self.alpha / D)
        W0 = math.sqrt(e_tii) * orthonormal_special(R, D, self.dtype, self.device)
        self.W = W0.unsqueeze(0).expand(self.G, R, D).contiguous()

    # -------------------------------------------------------------- public
    def precondition(self, X: torch.Tensor) -> torch.Tensor:
        """X: [G, N, dim] -> preconditioned, same shape (Frobenius norm preserved)."""
        return drive([self.precondition_gen(X)])[0]

    def precondition_gen(self, X: torch.Tensor, ip=None):
        """Generator form of ``precondition`` (yields Z, receives eigenpairs).  ``ip``:
        per-matrix |X|^2 when the caller already has it (HIP path); ``self.last_ip`` holds
        it afterwards (None on the PyTorch path)."""
        if self.t == 0:
            self._init_default()
            self.t = 1
            self.defer = False
            try:
                for _ in range(3):
                    yield from self._precondition_scaled(X, ip)
                    ip = self.last_ip
            finally:
                self.defer = True
            self.t = 0
        return (yield from self._precondition_scaled(X, ip))

    def _precondition_scaled(self, X, ip_in=None):
        if _fused_small_math(X, 1) and X.is_contiguous() and X.numel() % (4 * X.shape[0]) == 0:
            # HIP: |X|^2, |Y|^2 per matrix and the norm-preserving rescale + NaN guard in three
            # launches (+ one fill) instead of ~10 (csrc/kernels/ngd.hip).  |X|^2 is known
            # when X is the previous axis' (norm-preserved) output: ip_in, no extra pass.
            nat = _native.native()
            G, per = X.shape[0], X.numel() // X.shape[0]
            if ip_in is not None:
                ip = ip_in
                fp = torch.zeros(G, device=X.device, dtype=torch.float32)
            else:
                sums = torch.zeros(2, G, device=X.device, dtype=torch.float32)
                ip, fp = sums[0], sums[1]
                nat.ngd_sumsq(X.data_ptr(), per, G, ip.data_ptr(), _native.stream_ptr())
            self.last_ip = ip
            Y = yield from self._step(X, ip)
            Y = Y.contiguous()
            nat.ngd_sumsq(Y.data_ptr(), per, G, fp.data_ptr(), _native.stream_ptr())
            nat.ngd_rescale(X.data_ptr(), Y.data_ptr(), per, G, ip.data_ptr(), fp.data_ptr(), _native.stream_ptr())
            return Y
        ip = (X * X).sum(dim=(1, 2))
        self.last_ip = None
        Y = yield from self._step(X, ip)
        fp = (Y * Y).sum(dim=(1, 2))
        out = Y * torch.sqrt(ip / (fp + 1e-30)).view(-1, 1, 1)
        bad = torch.isnan(fp).view(-1, 1, 1)
        return torch.where(bad, X, out)

    def _step(self, X, trXX):
        updating = self._updating()
        self.t += 1
        W, d, rho = self.W, self.d, self.rho
        alpha, eta = self.alpha, self.eta
        R, D = self.rank, self.dim
        N = X.shape[1]
        H = torch.bmm(X, W.transpose(1, 2))                     # [G,N,R]
        Xh = torch.baddbmm(X, H, W, beta=1.0, alpha=-1.0)         # X - H W
        if not updating:
            return Xh
        J = torch.bmm(H.transpose(1, 2), X)                      # [G,R,D]
        if N > D:
            L = torch.bmm(J, W.transpose(1, 2))
        else:
            L = torch.bmm(H.transpose(1, 2), H)
        K = torch.bmm(J, J.transpose(1, 2))                      # [G,R,R]
        if _fused_small_math(X, R):
            yield from self._fused_update(J, K, L, trXX, N)
            return Xh
        dsum = d.sum(dim=1)                                       # [G]
        beta = rho * (1.0 + alpha) + alpha * dsum / D
        e = 1.0 / (beta.unsqueeze(1) / d + 1.0)
        ise = torch.rsqrt(e)                                      # 1/sqrt(e)
        zs = torch.clamp(torch.diagonal(K, dim1=1, dim2=2).sum(1), min=1.0)  # [G]
        drho = d + rho.unsqueeze(1)
        c1 = ((eta / N) ** 2) / zs
        c2 = ((eta / N) * (1.0 - eta)) / zs
        c3 = ((1.0 - eta) ** 2) / zs
        oo = ise.unsqueeze(2) * ise.unsqueeze(1)                  # outer(ise, ise)
        o1 = ise.unsqueeze(2) * (ise * drho).unsqueeze(1)         # outer(ise, ise*drho)
        Z = K * (c1.view(-1, 1, 1) * oo) + L * (c2.view(-1, 1, 1) * (o1 + o1.transpose(1, 2)))
        Z = Z + torch.diag_embed(c3.unsqueeze(1) * drho * drho)
        c, U = yield Z                                            # eigh, ascending
        c = c.flip(1)
        U = U.flip(2)
        c_floor = ((rho * (1.0 - eta)) ** 2) / zs
        c = torch.maximum(c, c_floor.unsqueeze(1))
        sqc = torch.sqrt(c) * torch.sqrt(zs).unsqueeze(1)
        rho1 = ((eta / N) * trXX + (1.0 - eta) * (D * rho + dsum) - sqc.sum(1)) / (D - R)
        floor = torch.clamp(DELTA * sqc.max(dim=1).values, min=EPSILON)
        d1 = torch.maximum(sqc - rho1.unsqueeze(1), floor.unsqueeze(1))
        rho1 = torch.maximum(rho1, floor)
        beta1 = rho1 * (1.0 + alpha) + alpha * d1.sum(1) / D
        e1 = 1.0 / (beta1.unsqueeze(1) / d1 + 1.0)
        wc = ((1.0 - eta) / (eta / N)) * drho
        B = J + wc.unsqueeze(2) * W
        lp = (eta / N) * torch.sqrt(e1) / sqc
        A = U.transpose(1, 2) * (lp.unsqueeze(2) * ise.unsqueeze(1))
        # in place: the state buffers keep their addresses, so a captured HIP graph of the
        # optimizer step reads and writes the same W / d / rho on every replay
        self.W.copy_(torch.bmm(A, B))
        self.d.copy_(d1)
        self.rho.copy_(rho1)
        return Xh

    def _fused_update(self, J, K, L, trXX, N):
        """The rank x rank math around the eigensolver in two HIP launches
        (csrc/kernels/ngd.hip), then W <- A (J + wc W) in place."""
        nat = _native.native()
        G, R, D = J.shape[0], self.rank, self.dim
        dev = J.device
        sp = _native.stream_ptr()
        Kc, Lc = K.contiguous(), L.contiguous()
        Z = torch.empty(G, R, R, device=dev, dtype=torch.float32)
        ise, drho = torch.empty(G, R, device=dev), torch.empty(G, R, device=dev)
        zs, dsum = torch.empty(G, device=dev), torch.empty(G, device=dev)
        nat.ngd_pre_eigh(Kc.data_ptr(), Lc.data_ptr(), self.d.data_ptr(), self.rho.data_ptr(), Z.data_ptr(),
                         ise.data_ptr(), drho.data_ptr(), zs.data_ptr(), dsum.data_ptr(), G, R, self.alpha, self.eta,
                         float(N), float(D), sp)
        post = (J, ise, drho, zs, dsum, trXX, N)
        if self.defer and DEFER:
            # the eigenpairs only shape this state's NEXT step: solved with every other
            # axis' Z in one launch at the end of the optimizer step (``drive``)
            yield Deferred(Z, lambda c, U: self._post_update(c, U, *post))
            return
        c, U = yield Z                                            # eigh, ascending
        self._post_update(c, U, *post)

    def _post_update(self, c, U, J, ise, drho, zs, dsum, trXX, N):
        nat = _native.native()
        G, R, D = J.shape[0], self.rank, self.dim
        dev = J.device
        A = torch.empty(G, R, R, device=dev, dtype=torch.float32)
        wc = torch.empty(G, R, device=dev, dtype=torch.float32)
        tr = trXX.contiguous()
        nat.ngd_post_eigh(c.contiguous().data_ptr(), U.contiguous().data_ptr(), ise.data_ptr(), drho.data_ptr(),
                          zs.data_ptr(), dsum.data_ptr(), tr.data_ptr(), self.d.data_ptr(), self.rho.data_ptr(),
                          A.data_ptr(), wc.data_ptr(), G, R, self.alpha, self.eta, float(N), float(D),
                          _native.stream_ptr())
        w_update(A, J, wc, self.W)                                # W <- A (J + wc W), in place

    # ------------------------------------------------- tiny-dim axes (HIP, no transposes)
    def small_ok(self, G: torch.Tensor) -> bool:
        """The kh / kw axes of 3x3 convs (dim <= 8): one streaming HIP pass per step instead of
        transpose + 2-5 badly shaped batched GEMMs (csrc/kernels/ngd.hip ngd_small_proj)."""
        return (_fused_small_math(G, self.rank) and hasattr(_native.native(), "ngd_small_proj")
                and _native.native().ngd_small_supported(self.dim, self.rank)
                and (G.numel() // G.shape[0]) % 4 == 0)

    def precondition_small_gen(self, G: torch.Tensor, A: int, B: int):
        """G: [P, A, dim, B] in its own (contiguous) layout -> preconditioned, same layout."""
        if self.t == 0:
            self._init_default()
            self.t = 1
            self.defer = False
            try:
                for _ in range(3):
                    yield from self._small_step(G, A, B)
            finally:
                self.defer = True
            self.t = 0
        return (yield from self._small_step(G, A, B))

    def _small_step(self, G, A, B):
        updating = self._updating()
        self.t += 1
        nat = _native.native()
        P, R, D = G.shape[0], self.rank, self.dim
        N = A * B
        nj = P * R * D if updating else 0
        # (every output is assigned by ngd_small_sums, none accumulated: no zero fill)
        buf = torch.empty(2 * P + nj + (P * R * R if updating else 0), device=G.device, dtype=torch.float32)
        sums = buf[:2 * P]
        ip, fp = sums[:P], sums[P:]
        J = buf[2 * P:2 * P + nj].view(P, R, D) if updating else None
        HH = buf[2 * P + nj:].view(P, R, R) if updating else None
        Y = torch.empty_like(G)
        part = torch.empty(nat.ngd_small_part_numel(P, A, D, B, R), device=G.device, dtype=torch.float32)
        nat.ngd_small_proj(G.data_ptr(), Y.data_ptr(), self.W.data_ptr(), P, A, D, B, R, sums.data_ptr(),
                           J.data_ptr() if updating else 0, HH.data_ptr() if updating else 0, part.data_ptr(),
                           _native.stream_ptr())
        self.last_ip = ip
        if updating:
            K, L = gram(J, self.W if N > D else None)
            L = HH if L is None else L
            yield from self._fused_update(J, K, L, ip, N)
        nat.ngd_rescale(G.data_ptr(), Y.data_ptr(), G.numel() // P, P, ip.data_ptr(), fp.data_ptr(),
                        _native.stream_ptr())
        return Y

    # ------------------------------------------------ general axes (HIP, no transposes)
    def proj_ok(self, G: torch.Tensor) -> bool:
        """Every other axis (dim >= 9, rank <= 80): one fused HIP pass per step in the
        parameter's own layout (csrc/kernels/ngd.hip ngd_proj: H = X W^T, X - H W, |X|^2,
        |Xh|^2 and, on update steps, J = H^T X and H^T H) instead of a transpose copy plus
        2-4 batched library GEMMs and two reductions."""
        return (_fused_small_math(G, self.rank) and hasattr(_native.native(), "ngd_proj")
                and _native.native().ngd_proj_supported(self.dim, self.rank)
                and (G.numel() // G.shape[0]) % 4 == 0)

    def precondition_proj_gen(self, G: torch.Tensor, A: int, B: int, ip=None):
        """G: [P, A, dim, B] contiguous -> preconditioned, same layout.  ``ip``: per-matrix
        |G|^2 when the previous axis already has it."""
        if self.t == 0:
            self._init_default()
            self.t = 1
            self.defer = False
            try:
                for _ in range(3):
                    yield from self._proj_step(G, A, B, ip)
                    ip = self.last_ip
            finally:
                self.defer = True
            self.t = 0
        return (yield from self._proj_step(G, A, B, ip))

    def _proj_step(self, G, A, B, ip_in):
        updating = self._updating()
        self.t += 1
        nat = _native.native()
        P, R, D = G.shape[0], self.rank, self.dim
        N = A * B
        need_hh = updating and N <= D  # L = H^T H (else J W^T, a [R, D] x [D, R] product)
        nj = P * R * D if updating else 0
        nh = P * R * R if need_hh else 0
        # (|X|^2, |Y|^2, J, H^T H are assigned by the fixed-order sum kernels: no zero fill)
        buf = torch.empty(2 * P + nj + nh, device=G.device, dtype=torch.float32)
        ip = ip_in if ip_in is not None else buf[:P]
        fp = buf[P:2 * P]
        J = buf[2 * P:2 * P + nj].view(P, R, D) if updating else None
        HH = buf[2 * P + nj:].view(P, R, R) if need_hh else None
        Y = torch.empty_like(G)
        Hb = torch.empty(nat.ngd_proj_hbuf_numel(P, A, D, B, R, ip_in is None, updating, need_hh), device=G.device,
                         dtype=torch.float32)
        sp = _native.stream_ptr()
        nat.ngd_proj(G.data_ptr(), Y.data_ptr(), self.W.data_ptr(), Hb.data_ptr(), P, A, D, B, R,
                     0 if ip_in is not None else ip.data_ptr(), fp.data_ptr(),
                     J.data_ptr() if updating else 0, HH.data_ptr() if need_hh else 0, sp)
        self.last_ip = ip
        if updating:
            K, L = gram(J, None if need_hh else self.W)
            L = HH if need_hh else L
            yield from self._fused_update(J, K, L, ip, N)
        nat.ngd_rescale(G.data_ptr(), Y.data_ptr(), G.numel() // P, P, ip.data_ptr(), fp.data_ptr(), sp)
        return Y

    def state_dict(self):
        return {"t": self.t, "W": self.W, "d": self.d, "rho": self.rho}

    def load_state_dict(self, sd):
        def mv(v):
            return v.to(self.device) if isinstance(v, torch.Tensor) else v
        W, d, rho = mv(sd["W"]), mv(sd["d"]), mv(sd["rho"])
        if isinstance(W, torch.Tensor):
            # the HIP kernels index W / d / rho by (G, rank, dim): a state saved for other
            # parameters (e.g. another rank's ZeRO-2 shard) must not be loaded
            want = {"W": (self.G, self.rank, self.dim), "d": (self.G, self.rank), "rho": (self.G,)}
            for k, v in (("W", W), ("d", d), ("rho", rho)):
                if not isinstance(v, torch.Tensor) or tuple(v.shape) != want[k]:
                    got = tuple(v.shape) if isinstance(v, torch.Tensor) else type(v).__name__
                    raise ValueError(f"NGD state {k}: shape {got}, expected {want[k]}")
        self.t = int(sd["t"])
        self.W, self.d, self.rho = W, d, rho
        if isinstance(self.W, torch.Tensor):  # own (contiguous) buffers: updated in place later
            self.W, self.d, self.rho = self.W.clone(), self.d.clone(), self.rho.clone()


class OnlineNaturalGradient:
    """Single-tensor API twin of the reference class (one axis of one parameter);
    backed by the batched state with G = 1."""

    def __init__(self, params, axis, alpha=4.0, rank=-1, update_period=4, eta=0.1):
        assert 0 <= axis < len(params.shape)
        assert 0 < eta < 1 and update_period > 0
        self.axis = axis
        self.dim = params.shape[axis]
        self.noop = self.dim == 1
        self.rank = default_rank(self.dim, rank) if not self.noop else 0
        self.state = None if self.noop else NGState(1, self.dim, self.rank, alpha, update_period, eta, params.dtype,
                                                    params.device)

    @property
    def t(self):
        return 0 if self.state is None else self.state.t

    def precondition_directions(self, deriv):
        if self.noop:
            return deriv
        X = deriv.transpose(-1, self.axis).contiguous()
        shp = X.shape
        Y = self.state.precondition(X.view(1, -1, self.dim))
        return Y.view(shp).transpose(-1, self.axis)


def _group_view(grad, slots):
    """The stacked [G, *shape] gradients of a shape group as a VIEW of the flat gradient when
    its slots sit back to back without padding (models can ask for that: utils/flat.py
    ``flat_adjacent``), else None (the caller stacks copies)."""
    s0 = slots[0]
    n = s0.numel
    for i, s in enumerate(slots):
        if s.offset != s0.offset + i * n or tuple(s.shape) != tuple(s0.shape):
            return None
    return grad[s0.offset:s0.offset + n * len(slots)].view(len(slots), *s0.shape)


class _ShapeGroup:
    def __init__(self, shape, params, alpha, rank, update_period, eta, dtype, device):
        self.shape = tuple(shape)
        self.params = params
        self.axes = []
        for ax, dim in enumerate(self.shape):
            if dim > 1:
                r = default_rank(dim, rank if (rank >= 0 and rank < dim) else -1)
                self.axes.append((ax, NGState(len(params), dim, r, alpha, update_period, eta, dtype, device)))

    def precondition(self, G: torch.Tensor) -> torch.Tensor:
        """G: [P, *shape] stacked gradients -> preconditioned (same layout)."""
        return drive([self.precondition_gen(G)])[0]

    def precondition_gen(self, G: torch.Tensor):
        # every axis preserves each matrix's Frobenius norm, so |G|^2 measured by the first
        # (HIP) axis is handed on instead of re-reduced per axis
        ip = None
        for ax, st in self.axes:
            a = ax + 1  # leading stack dim
            if st.small_ok(G):
                G = G.contiguous()
                A = math.prod(self.shape[:ax])
                B = math.prod(self.shape[ax + 1:])
                G = (yield from st.precondition_small_gen(G, A, B)).view(G.shape)
            elif st.proj_ok(G):
                G = G.contiguous()
                A = math.prod(self.shape[:ax])
                B = math.prod(self.shape[ax + 1:])
                G = (yield from st.precondition_proj_gen(G, A, B, ip)).view(G.shape)
            else:
                X = G.transpose(-1, a).contiguous()
                shp = X.shape
                Y = yield from st.precondition_gen(X.view(shp[0], -1, shp[-1]), ip)
                G = Y.view(shp).transpose(-1, a)
            ip = st.last_ip
        return G


class NGD(SGD):
    """NGD optimizer (``ngd_optimizer.py:423-508``) over a flat parameter buffer.

    step: g <- g*clip_coef + wd*p (in place in the flat grad) -> per-axis natural-
    gradient preconditioning of every parameter (batched by shape) written back into
    the flat grad -> fused SGD momentum/nesterov update (wd already applied)."""

    def __init__(self, flat: FlatParams, lr=1e-4, momentum=0, dampening=0, weight_decay=0, nesterov=False,
                 ngd=True, alpha=4, rank=-1, update_period=4, eta=0.1, overlap_eigh=True, **kw):
        if lr < 0.0:
            raise ValueError(f"Invalid learning rate: {lr}")
        if momentum < 0.0:
            raise ValueError(f"Invalid momentum value: {momentum}")
        if weight_decay < 0.0:
            raise ValueError(f"Invalid weight_decay value: {weight_decay}")
        super().__init__(flat, lr=lr, momentum=momentum, dampening=dampening, weight_decay=weight_decay,
                         nesterov=nesterov, **kw)
        self.group.update(ngd=ngd, alpha=alpha, rank=rank, update_period=update_period, eta=eta)
        self.groups = None
        # deferred eigensolves on a side stream, overlapping the next step (see drive);
        # FDT_NGD_OVERLAP=0: solved inline on the caller's stream instead (A/B: beside the next
        # step's library GEMMs the one-workgroup-per-matrix solver delays them,
        # profiles/r4/probe_side_eigh.txt)
        self.overlap_eigh = overlap_eigh and os.environ.get("FDT_NGD_OVERLAP", "1") != "0"
        self._side = None
        self._pending = None
        self.graphs = GRAPHS
        self._gcache = {}
        self._gpool = None
        self.graph_replays = 0
        self.lr_dev = None

    def _build_groups(self):
        g = self.group
        by_shape = {}
        for s in self.flat.slots:
            by_shape.setdefault(tuple(s.shape), []).append(s)
        self.groups = [
            (_ShapeGroup(shape, slots, g["alpha"], g["rank"], g["update_period"], g["eta"], self.flat.data.dtype,
                         self.flat.device), slots)
            for shape, slots in by_shape.items()]

    def _side_stream(self, grad):
        """Stream for the deferred eigensolve + state update (see ``drive``): CUDA only."""
        if not (self.overlap_eigh and grad.is_cuda):
            return None
        if self._side is None:
            self._side = torch.cuda.Stream(device=grad.device)
        return self._side

    def sync_state(self):
        """Order the caller's stream after the previous step's deferred state update (the
        next preconditioning step, checkpointing and tests read W / d / rho)."""
        if self._pending is not None:
            done, _keep = self._pending
            torch.cuda.current_stream().wait_event(done)
            self._pending = None

    def _scale_deferrable(self, grad_scale) -> bool:
        """On a step where no preconditioner updates (and without weight decay) the whole
        preconditioning is homogeneous of degree one in the gradient -- fixed projections, then
        a norm-preserving rescale -- so the clip coefficient can be applied by the final SGD
        kernel (it reads the coefficient anyway) instead of by a separate pass over the flat
        gradient before it: NGD(c g) = c NGD(g).  Update steps fold g into the Fisher estimate
        and keep the reference order."""
        if grad_scale is None or not DEFER_SCALE or self.group["weight_decay"] != 0 or not self.group["ngd"]:
            return False
        sts = [st for sg, _ in (self.groups or []) for _, st in sg.axes]
        return bool(sts) and not any(st._updating() for st in sts)

    def _precondition(self, grad, grad_scale, defer_out=None):
        """grad <- NGD-preconditioned (grad * scale + wd * p), in place.  ``defer_out``: collect
        the deferred eigensolves instead of running them (graph capture).  Returns True when
        the scale was left to the SGD kernel (``_scale_deferrable``)."""
        self.sync_state()
        g = self.group
        deferred_scale = self._scale_deferrable(grad_scale)
        if grad_scale is not None and not deferred_scale:
            grad.mul_(grad_scale)
        if g["weight_decay"] != 0:
            grad.add_(self.flat.data, alpha=g["weight_decay"])
        if g["ngd"]:
            if self.groups is None:
                self._build_groups()
            live = [(sg, slots) for sg, slots in self.groups if sg.axes]
            views = [_group_view(grad, slots) for _, slots in live]
            gens = [sg.precondition_gen(v if v is not None else
                                        torch.stack([grad[s.offset:s.offset + s.numel].view(s.shape) for s in slots]))
                    for (sg, slots), v in zip(live, views)]
            side = self._side_stream(grad)
            if defer_out is not None:
                outs = drive(gens, defer_out=defer_out)
            elif side is not None:
                outs, self._pending = drive(gens, side)
            else:
                outs = drive(gens)
            dst, src = [], []
            for (sg, slots), out, v in zip(live, outs, views):
                if v is not None:
                    if out.data_ptr() != v.data_ptr():
                        v.copy_(out)  # one contiguous copy per shape group
                    continue
                for i, s in enumerate(slots):
                    dst.append(grad[s.offset:s.offset + s.numel].view(s.shape))
                    src.append(out[i])
            if dst:
                torch._foreach_copy_(dst, src)  # multi-tensor launches, not one copy per parameter
        return deferred_scale

    @torch.no_grad()
    def _step(self, grad_scale, found_inf, d_override=None):
        if found_inf is not None and bool(found_inf.item() != 0):
            if self.zero_grad_in_step:  # GradScaler skip (fp16 mode only); still clear the gradient
                self.flat.grad.zero_()
            return
        if self._graph_ready(grad_scale, found_inf, d_override):
            return self._graph_step(grad_scale)
        self._eager_step(grad_scale)

    def _eager_step(self, grad_scale, defer_out=None):
        g = self.group
        if self.lr_dev is not None and not torch.cuda.is_current_stream_capturing():
            self._fill_hp()  # (the SGD kernel reads [lr, momentum] from it once graphs exist)
        deferred_scale = self._precondition(self.flat.grad, grad_scale, defer_out)
        wd = g["weight_decay"]
        g["weight_decay"] = 0.0
        try:
            super()._step(grad_scale if deferred_scale else None, None)
        finally:
            g["weight_decay"] = wd

    # ------------------------------------------------------------ HIP-graph steps
    # After the initialisation schedule (every preconditioner updates on each of its first 10
    # calls) the step is periodic: update iff t % update_period == 0, the same for every
    # state (they advance together).  Each kind of step -- update / plain -- is captured once
    # and replayed: ~100-200 launches become one graph launch (+ one for the deferred
    # eigensolve).  Everything a replay needs is static: gradients / parameters / momentum in
    # the flat buffers, W / d / rho updated in place, the clip coefficient and the learning
    # rate read from device buffers (``lr_dev``: schedulers keep working).  Host-side values
    # baked into a capture are part of the cache key (momentum, dampening, weight decay, ...).
    #
    # The deferred eigensolve + W / d / rho update of an update step is its OWN graph,
    # replayed on the side stream after the main graph, and the next step waits on an event
    # recorded AFTER that replay.  (Round-2 root cause of the 2-4 % replay drift: the side-
    # stream work had been captured into the step's graph with its completion event recorded
    # during capture; an event recorded inside a capture is not re-recorded by replays, so the
    # next step's wait on it returned at once and its preconditioning read W / d / rho while
    # the previous replay was still rewriting them.)
    def _graph_states(self):
        return [st for sg, _ in (self.groups or []) for _, st in sg.axes]

    def _graph_ready(self, grad_scale, found_inf, d_override):
        g = self.group
        if not (self.graphs and g["ngd"] and self.flat.data.is_cuda and _native.enabled() and d_override is None
                and found_inf is None and self.groups is not None and _native_eigh(self.flat.device)):
            return False
        if torch.cuda.is_current_stream_capturing():
            return False
        sts = self._graph_states()
        if not sts or min(st.t for st in sts) < 10 or len({(st.t, st.update_period) for st in sts}) != 1:
            return False
        if g["momentum"] != 0 and not self.state.get("__flat__", {}).get("initialized", 0):
            return False
        return True

    def _graph_key(self, grad_scale):
        g = self.group
        st = self._graph_states()[0]
        upd = st.t % st.update_period == 0
        # lr and momentum are read from ``lr_dev`` by the kernel (OneCycleLR cycles both every
        # step); only whether momentum is on (a momentum buffer in the capture) is baked
        plan = self._pack_plan()
        return (upd, g["momentum"] != 0, float(g["dampening"]), float(g["weight_decay"]), bool(g["nesterov"]),
                0 if grad_scale is None else grad_scale.data_ptr(), getattr(plan, "upd_gen", 0))

    def _fill_hp(self):
        g = self.group
        self.lr_dev[0].fill_(float(g["lr"]))  # (two scalar fills: no pageable host copy)
        self.lr_dev[1].fill_(float(g["momentum"]))

    def _graph_step(self, grad_scale):
        key = self._graph_key(grad_scale)
        if self.lr_dev is None:
            self.lr_dev = torch.zeros(2, device=self.flat.device, dtype=torch.float32)  # [lr, momentum]
        self._fill_hp()
        ent = self._gcache.get(key)
        if ent is None:
            # graphs of an older pack-table generation hold freed table / layout addresses
            for k in [k for k, e in self._gcache.items() if e.get("packed") and k[-1] != key[-1]]:
                del self._gcache[k]
            ent = self._gcache[key] = self._capture(grad_scale)
        self.sync_state()  # the previous update's side-stream graph -> before this replay
        ent["main"].replay()
        self._packed = ent.get("packed", False)  # (the captured SGD tail's fused conv repack)
        if ent["side"] is not None:
            cur = torch.cuda.current_stream()
            side = self._side_stream(self.flat.grad) or cur
            side.wait_stream(cur)
            with torch.cuda.stream(side):
                ent["side"].replay()
                done = torch.cuda.Event()
                done.record(side)
            self._pending = (done, None)
        for st in self._graph_states():
            st.t += 1
        self.graph_replays += 1

    def _capture(self, grad_scale):
        """Capture one step kind: the main graph (preconditioning + momentum update) and, on
        update steps, the deferred eigensolves + state updates as a second graph."""
        from ..ops.eigh import NGD_TOL, eigh_many
        from ..parallel.graphs import capture_guard
        self.sync_state()
        dev = self.flat.device
        if self._gpool is None:
            self._gpool = torch.cuda.graph_pool_handle()
        sts = self._graph_states()
        t0 = [st.t for st in sts]
        cur = torch.cuda.current_stream()
        cs = torch.cuda.Stream(device=dev)
        cs.wait_stream(cur)
        torch.cuda.synchronize(dev)
        deferred = []
        main = torch.cuda.CUDAGraph()
        side_g = None
        try:
            with torch.cuda.stream(cs):
                with torch.cuda.graph(main, pool=self._gpool, stream=cs, capture_error_mode="thread_local"), \
                        capture_guard():
                    self._eager_step(grad_scale, defer_out=deferred)
                if deferred:
                    side_g = torch.cuda.CUDAGraph()
                    with torch.cuda.graph(side_g, pool=self._gpool, stream=cs, capture_error_mode="thread_local"), \
                            capture_guard():
                        for d, (c, U) in zip(deferred, eigh_many([d.Z for d in deferred], tol=NGD_TOL)):
                            d.fn(c, U)
        finally:
            for st, t in zip(sts, t0):  # the captures ran the host schedule once: undo it
                st.t = t
        cur.wait_stream(cs)
        return {"main": main, "side": side_g, "keep": deferred, "packed": getattr(self, "_packed", False)}

    def _states(self):
        """Every batched per-axis preconditioner state (empty before the first step)."""
        self.sync_state()
        if self.groups is None:
            return []
        return [st for sg, _ in self.groups for _, st in sg.axes]

    def ngd_state_dict(self):
        self.sync_state()
        if self.groups is None:
            return []
        return [[st.state_dict() for _, st in sg.axes] for sg, _ in self.groups]

    def load_ngd_state_dict(self, sd):
        """Restore per-axis preconditioner states saved by ``ngd_state_dict`` (same model)."""
        self.sync_state()
        if not sd:
            return
        if self.groups is None:
            self._build_groups()
        if len(sd) != len(self.groups):
            raise ValueError("NGD state was saved for a different model")
        for (sg, _), axes_sd in zip(self.groups, sd):
            for (_, st), s in zip(sg.axes, axes_sd):
                st.load_state_dict(s)
