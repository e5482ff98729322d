"""HIP kernel numerics vs plain-PyTorch fp32 references (run on an MI355X: -m gpu)."""
import math

import pytest
import numpy as np
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def rel(a, b):
    a, b = a.float(), b.float()
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


# ---------------------------------------------------------------- optimizers
@pytest.mark.parametrize("kind", ["sgd", "madgrad", "mirror", "adam"])
def test_flat_optimizers_match_cpu(cuda, kind):
    from faster_distributed_training_amd.optim import flat_optim as O
    from faster_distributed_training_amd.utils.flat import FlatParams
    torch.manual_seed(0)
    nets = [torch.nn.Sequential(torch.nn.Linear(33, 17), torch.nn.Linear(17, 5)) for _ in range(2)]
    nets[1].load_state_dict(nets[0].state_dict())
    fg = FlatParams(nets[0].to(cuda), device=cuda)
    fc = FlatParams(nets[1], device="cpu")
    mk = {"sgd": lambda f: O.SGD(f, lr=0.1, momentum=0.9, weight_decay=1e-3, nesterov=True),
          "madgrad": lambda f: O.MADGRAD(f, lr=0.05, momentum=0.9, weight_decay=1e-4),
          "mirror": lambda f: O.MirrorMADGRAD(f, lr=0.05, momentum=0.9),
          "adam": lambda f: O.Adam(f, lr=1e-2, weight_decay=1e-2, adamw=True)}[kind]
    og, oc = mk(fg), mk(fc)
    for step in range(5):
        g = torch.randn(fg.numel)
        fg.grad.copy_(g.to(cuda))
        fc.grad.copy_(g)
        coef = torch.tensor([0.7])
        og.step(grad_scale=coef.to(cuda))
        oc.step(grad_scale=coef)
    assert rel(fg.data.cpu(), fc.data) < 1e-5


@pytest.mark.parametrize("kind", ["sgd", "madgrad", "mirror", "adam"])
def test_skipped_step_clears_gradient(cuda, kind):
    """found_inf set (non-finite gradients): the kernel leaves parameters and optimizer
    state untouched but still zeroes the gradient, so the next step starts clean."""
    from faster_distributed_training_amd.optim import flat_optim as O
    from faster_distributed_training_amd.utils.flat import FlatParams
    torch.manual_seed(1)
    f = FlatParams(torch.nn.Linear(40, 24).to(cuda), device=cuda)
    opt = {"sgd": lambda: O.SGD(f, lr=0.1, momentum=0.9), "madgrad": lambda: O.MADGRAD(f, lr=0.05),
           "mirror": lambda: O.MirrorMADGRAD(f, lr=0.05), "adam": lambda: O.Adam(f, lr=1e-2)}[kind]()
    f.grad.copy_(torch.randn(f.numel, device=cuda))
    opt.step()
    before = f.data.clone()
    f.grad.fill_(float("nan"))
    found = torch.ones(1, device=cuda, dtype=torch.int32)
    opt.step(found_inf=found)
    torch.cuda.synchronize()
    assert torch.equal(f.data, before)
    assert torch.count_nonzero(f.grad).item() == 0


def test_grad_clipper(cuda):
    from faster_distributed_training_amd.optim.flat_optim import GradClipper
    from faster_distributed_training_amd.utils.flat import FlatParams
    net = torch.nn.Linear(300, 300).to(cuda)
    f = FlatParams(net, device=cuda)
    f.grad.normal_()
    c = GradClipper(f)
    norm = c(1.0)
    ref = f.grad.double().norm()
    assert abs(float(norm) - float(ref)) / float(ref) < 1e-5
    assert abs(float(c.coef) - 1.0 / (float(ref) + 1e-6)) < 1e-6


# ---------------------------------------------------------------- mixup
def test_mixup_kernels(cuda):
    from faster_distributed_training_amd.ops.mixup import mixup_cross_entropy, mixup_interpolate
    x = torch.randn(16, 3, 8, 8, device=cuda, requires_grad=True)
    perm = torch.randperm(16, device=cuda)
    lam = torch.rand(16, device=cuda, requires_grad=True)
    out = mixup_interpolate(x, perm, lam)
    g = torch.randn_like(out)
    out.backward(g)
    x2 = x.detach().clone().requires_grad_()
    lam2 = lam.detach().clone().requires_grad_()
    l4 = lam2.view(16, 1, 1, 1)
    ref = l4 * x2 + (1 - l4) * x2[perm]
    ref.backward(g)
    assert rel(out, ref) < 1e-6 and rel(x.grad, x2.grad) < 1e-6 and rel(lam.grad, lam2.grad) < 1e-5
    logits = torch.randn(64, 10, device=cuda, requires_grad=True)
    ya, yb = torch.randint(0, 10, (64,), device=cuda), torch.randint(0, 10, (64,), device=cuda)
    lv = torch.rand(64, device=cuda)
    loss = mixup_cross_entropy(logits, ya, yb, lv)
    loss.backward()
    l2 = logits.detach().clone().requires_grad_()
    ref = (lv * F.cross_entropy(l2, ya, reduction="none") + (1 - lv) * F.cross_entropy(l2, yb, reduction="none")).mean()
    ref.backward()
    assert abs(loss.item() - ref.item()) < 1e-5 and rel(logits.grad, l2.grad) < 1e-5
    # int32 labels take the conversion path, int64 are read directly: same result
    l3 = logits.detach().clone().requires_grad_()
    loss32 = mixup_cross_entropy(l3, ya.int(), yb.int(), lv)
    loss32.backward()
    assert loss32.item() == loss.item() and torch.equal(l3.grad, logits.grad)
    # one lambda for the batch as a python float (no lambda vector) == the same value per sample
    l5, l6 = logits.detach().clone().requires_grad_(), logits.detach().clone().requires_grad_()
    ls = mixup_cross_entropy(l5, ya, yb, 0.3)
    lt = mixup_cross_entropy(l6, ya, yb, torch.full((64,), 0.3, device=cuda))
    (ls * 2).backward()
    (lt * 2).backward()
    assert ls.item() == lt.item() and torch.equal(l5.grad, l6.grad)


@pytest.mark.gpu
@pytest.mark.parametrize("b", [128, 1024])
def test_mixup_ce_fp16_loss_scaled(cuda, b):
    """fp16 logits under a 65536 loss scale: the fused CE's d(logits) is scaled before it is
    rounded to fp16: equals F.cross_entropy's fp32 gradient scaled then cast."""
    from faster_distributed_training_amd.ops.mixup import mixup_cross_entropy
    torch.manual_seed(0)
    base = (torch.randn(b, 10, device=cuda) * 4).half()
    ya, yb = torch.randint(0, 10, (b,), device=cuda), torch.randint(0, 10, (b,), device=cuda)
    lv = torch.rand(b, device=cuda)
    scale = 65536.0
    lg = base.clone().requires_grad_()
    loss = mixup_cross_entropy(lg, ya, yb, lv)
    (loss * scale).backward()
    assert lg.grad.dtype == torch.float16
    l2 = base.float().requires_grad_()
    ref = (lv * F.cross_entropy(l2, ya, reduction="none") + (1 - lv) * F.cross_entropy(l2, yb, reduction="none")).mean()
    (ref * scale).backward()
    want = l2.grad.half()
    assert abs(loss.item() - ref.item()) < 1e-4
    # the small entries survive: no more flushed-to-zero gradients than the reference has
    assert int((lg.grad == 0).sum()) <= int((want == 0).sum())
    assert rel(lg.grad.float(), want.float()) < 2e-3


@pytest.mark.parametrize("b", [1, 7, 128, 1000, 1024])
def test_mixup_prep_kernel(cuda, b):
    """mixup_data's one-kernel device path: a valid permutation (every index once), the
    permuted labels, the lambda vector; different host seeds give different permutations,
    the same generator state the same one; the mixed batch equals lam*x + (1-lam)*x[perm]."""
    from faster_distributed_training_amd.ops.mixup import mixup_data
    x = torch.randn(b, 3, 4, 4, device=cuda)
    y = torch.randint(0, 10, (b,), device=cuda)
    g = torch.Generator().manual_seed(3)
    mixed, ya, yb, lam = mixup_data(x, y, alpha=0.99, generator=g)
    assert ya is y and yb.dtype == torch.int64
    # recover the permutation from the labels' source rows: x rows are distinct
    d = ((mixed - lam * x).reshape(b, -1).unsqueeze(1) - (1 - lam) * x.reshape(1, b, -1)).abs().amax(-1)
    perm = d.argmin(1)
    assert torch.equal(perm.sort().values, torch.arange(b, device=cuda))
    assert torch.equal(yb, y[perm])
    ref = lam * x + (1 - lam) * x[perm]
    assert rel(mixed, ref) < 1e-6
    g2 = torch.Generator().manual_seed(3)
    m2, _, yb2, lam2 = mixup_data(x, y, alpha=0.99, generator=g2)
    assert lam2 == lam and torch.equal(m2, mixed) and torch.equal(yb2, yb)
    if b >= 128:
        m3, _, _, _ = mixup_data(x, y, alpha=0.99, generator=g2)
        assert not torch.equal(m3, mixed)


@pytest.mark.parametrize("C", [10, 100])
def test_mixup_ce_fused_meter(cuda, C):
    """The loss kernel's fused accuracy/loss accumulation equals DeviceMeter's own update
    (argmax first occurrence, lambda-weighted correct, samples), over two steps."""
    from faster_distributed_training_amd.ops.mixup import mixup_cross_entropy
    from faster_distributed_training_amd.train.metrics import DeviceMeter
    fused, plain = DeviceMeter(cuda), DeviceMeter(cuda)
    for step in range(2):
        logits = torch.randn(96, C, device=cuda).to(torch.bfloat16)
        logits[:8] = 0.0  # ties: argmax must pick the first index
        ya, yb = torch.randint(0, C, (96,), device=cuda), torch.randint(0, C, (96,), device=cuda)
        lv = torch.rand(96, device=cuda)
        loss = mixup_cross_entropy(logits, ya, yb, lv, meter=fused)
        assert fused.fused
        ref = (lv * F.cross_entropy(logits.float(), ya, reduction="none")
               + (1 - lv) * F.cross_entropy(logits.float(), yb, reduction="none")).mean()
        assert abs(loss.item() - ref.item()) < 1e-4
        fused.update(loss, logits, ya, yb, lv)
        plain.update(loss, logits, ya, yb, lv)
    assert fused.steps == plain.steps == 2
    assert rel(fused.acc, plain.acc) < 1e-5, (fused.acc, plain.acc)


# ---------------------------------------------------------------- transformer ops
@pytest.mark.parametrize("d,dt", [(512, torch.float32), (512, torch.bfloat16), (256, torch.float32)])
def test_layernorm(cuda, d, dt):
    from faster_distributed_training_amd.ops.layernorm import _LayerNormNative, layer_norm_reference
    x = (torch.randn(3, 37, d, device=cuda) * 2 + 0.5).to(dt).requires_grad_()
    a = (torch.rand(d, device=cuda) + 0.5).requires_grad_()
    b = torch.randn(d, device=cuda).requires_grad_()
    y = _LayerNormNative.apply(x, a, b, 1e-6, dt)
    g = torch.randn_like(y)
    y.backward(g)
    x2, a2, b2 = [t.detach().float().clone().requires_grad_() for t in (x, a, b)]
    ref = layer_norm_reference(x2, a2, b2, 1e-6)
    ref.backward(g.float())
    tol = 1e-5 if dt == torch.float32 else 2e-2
    assert rel(y, ref) < tol
    assert rel(x.grad, x2.grad) < max(tol, 1e-4)
    assert rel(a.grad, a2.grad) < max(tol, 1e-4) and rel(b.grad, b2.grad) < max(tol, 1e-4)


def test_embedding(cuda):
    from faster_distributed_training_amd.ops.embedding import _EmbeddingNative, embedding_sum_reference
    V, d, B, L = 1000, 512, 4, 33
    tw = torch.randn(V, d, device=cuda, requires_grad=True)
    pw = torch.randn(512, d, device=cuda, requires_grad=True)
    sw = torch.randn(3, d, device=cuda, requires_grad=True)
    ids = torch.randint(0, V, (B, L), device=cuda)
    ty = torch.randint(0, 2, (B, L), device=cuda)
    pos = torch.arange(512, device=cuda)
    out = _EmbeddingNative.apply(ids, ty, pos, tw, pw, sw, math.sqrt(d))
    g = torch.randn_like(out)
    out.backward(g)
    t2, p2, s2 = [w.detach().clone().requires_grad_() for w in (tw, pw, sw)]
    ref = embedding_sum_reference(ids, ty, pos, t2, p2, s2, math.sqrt(d))
    ref.backward(g)
    assert rel(out, ref) < 1e-6
    assert rel(tw.grad, t2.grad) < 1e-5 and rel(pw.grad, p2.grad) < 1e-5 and rel(sw.grad, s2.grad) < 1e-5


def test_embedding_bwd_padding_heavy(cuda):
    """Backward with a heavily repeated (padding) token whose rows carry zero gradient, many
    rows per segment id and several workgroups (LDS segment path + position reduction)."""
    from faster_distributed_training_amd.ops.embedding import _EmbeddingNative, embedding_sum_reference
    V, d, B, L = 300, 512, 9, 40
    tw = torch.randn(V, d, device=cuda, requires_grad=True)
    pw = torch.randn(512, d, device=cuda, requires_grad=True)
    sw = torch.randn(3, d, device=cuda, requires_grad=True)
    ids = torch.randint(1, V, (B, L), device=cuda)
    ids[:, 25:] = 0  # padding token
    ty = torch.randint(0, 3, (B, L), device=cuda)
    pos = torch.arange(512, device=cuda)
    out = _EmbeddingNative.apply(ids, ty, pos, tw, pw, sw, math.sqrt(d))
    g = torch.randn_like(out)
    g[:, 25:] = 0.0  # masked positions: no gradient
    g[0, 3] = 0.0
    out.backward(g)
    t2, p2, s2 = [w.detach().clone().requires_grad_() for w in (tw, pw, sw)]
    embedding_sum_reference(ids, ty, pos, t2, p2, s2, math.sqrt(d)).backward(g)
    assert rel(tw.grad, t2.grad) < 1e-5 and rel(pw.grad, p2.grad) < 1e-5 and rel(sw.grad, s2.grad) < 1e-5


def test_fused_mlp(cuda):
    from faster_distributed_training_amd.ops.mlp import fused_mlp
    X = torch.randn(64, 512, device=cuda, requires_grad=True)
    W1 = torch.randn(1024, 512, device=cuda, requires_grad=True) * 0.05
    W1 = W1.detach().requires_grad_()
    b1 = torch.randn(1, 1024, device=cuda, requires_grad=True)
    W2 = (torch.randn(4, 1024, device=cuda) * 0.05).requires_grad_()
    b2 = torch.randn(1, 4, device=cuda, requires_grad=True)
    out = fused_mlp(X, W1, b1, W2, b2)
    g = torch.randn_like(out)
    out.backward(g)
    ts = [t.detach().clone().requires_grad_() for t in (X, W1, b1, W2, b2)]
    ref = F.linear(torch.relu(F.linear(ts[0], ts[1], ts[2][0])), ts[3], ts[4][0])
    ref.backward(g)
    assert rel(out, ref) < 1e-5
    for a, b in zip((X, W1, b1, W2, b2), ts):
        assert rel(a.grad, b.grad) < 1e-4


def test_augment_matches_cpu(cuda):
    from faster_distributed_training_amd.data.cifar import DeviceCIFARLoader, synthetic_cifar
    data, tg = synthetic_cifar(64, seed=3)
    ld = DeviceCIFARLoader(data, tg, 64, cuda, train=False, shuffle=False, drop_last=False, out_dtype=torch.float32)
    x, y = next(iter(ld))
    from faster_distributed_training_amd.data.cifar import augment_cpu
    ref = augment_cpu(torch.from_numpy(data), train=False)
    assert rel(x.float().cpu(), ref) < 1e-6
    assert torch.equal(y.cpu(), torch.from_numpy(tg).long())
    ld2 = DeviceCIFARLoader(data, tg, 64, cuda, train=True, shuffle=False, drop_last=False, out_dtype=torch.float32)
    xa, _ = next(iter(ld2))
    # each augmented image is a crop/flip of the normalised original: same value multiset
    # on the interior is hard to check exactly; check statistics + range instead
    assert xa.shape == (64, 3, 32, 32)
    assert torch.isfinite(xa).all()


@pytest.mark.parametrize("order", [("crop", "flip", "normalize"), ("normalize", "crop", "flip")])
def test_augment_padding_follows_transform_order(cuda, order):
    """Faithful transform permutation (Q13): normalising before the padded crop pads with 0
    in normalised space, otherwise with raw 0 (= -mean/std)."""
    from faster_distributed_training_amd.data.cifar import CIFAR_MEAN, CIFAR_STD, DeviceCIFARLoader
    data = np.full((256, 32, 32, 3), 128, dtype=np.uint8)
    tg = np.zeros(256, dtype=np.int64)
    ld = DeviceCIFARLoader(data, tg, 256, cuda, train=True, shuffle=False, out_dtype=torch.float32, order=order)
    x, _ = next(iter(ld))
    x = x.cpu()
    for c in range(3):
        inside = (128 / 255 - CIFAR_MEAN[c]) / CIFAR_STD[c]
        pad = 0.0 if order[0] == "normalize" else -CIFAR_MEAN[c] / CIFAR_STD[c]
        v = x[:, c]
        is_in = (v - inside).abs() < 1e-5
        is_pad = (v - pad).abs() < 1e-5
        assert bool((is_in | is_pad).all())
        assert 0 < int(is_pad.sum()) < v.numel() // 4  # some crops reach into the padding


@pytest.mark.parametrize("n,G", [(2, 5), (5, 3), (32, 4), (64, 2), (80, 8), (1, 2), (127, 1)])
def test_jacobi_eigh_matches_fp64_lapack(cuda, n, G):
    from faster_distributed_training_amd.ops.eigh import batched_eigh
    torch.manual_seed(n)
    B = torch.randn(G, n, n, device=cuda)
    Z = B @ B.transpose(1, 2) / n + torch.diag_embed(torch.rand(G, n, device=cuda))
    Z[0] = Z[0] * 1e3  # scale invariance
    w, V = batched_eigh(Z)
    wr, Vr = torch.linalg.eigh(Z.double().cpu())
    assert torch.allclose(w.double().cpu(), wr, rtol=1e-4, atol=1e-4 * wr.abs().max().item())
    # reconstruction and orthonormality (eigenvectors are unique only up to sign/rotation)
    Zr = V @ torch.diag_embed(w) @ V.transpose(1, 2)
    assert rel(Zr, Z) < 1e-5
    eye = torch.eye(n, device=cuda).expand(G, n, n)
    assert rel(V.transpose(1, 2) @ V, eye) < 1e-5


def test_jacobi_eigh_degenerate_and_diagonal(cuda):
    from faster_distributed_training_amd.ops.eigh import batched_eigh
    Z = torch.diag_embed(torch.tensor([[3.0, 1.0, 1.0, 2.0]], device=cuda))
    w, V = batched_eigh(Z)
    assert torch.allclose(w, torch.tensor([[1.0, 1.0, 2.0, 3.0]], device=cuda))
    assert rel(V @ torch.diag_embed(w) @ V.transpose(1, 2), Z) < 1e-6


def test_jacobi_eigh_ragged_one_launch(cuda):
    """eigh_many: matrices of different sizes (NGD shape groups) in one ragged launch."""
    from faster_distributed_training_amd.ops.eigh import eigh_many
    torch.manual_seed(1)
    Zs = []
    for G, n in [(3, 80), (2, 5), (4, 32), (1, 64)]:
        B = torch.randn(G, n, 3, device=cuda)
        Zs.append(B @ B.transpose(1, 2) + 1e-3 * torch.eye(n, device=cuda))  # NGD-like: low rank + ridge
    outs = eigh_many(Zs)
    for Z, (w, V) in zip(Zs, outs):
        wr = torch.linalg.eigvalsh(Z.double().cpu())
        assert torch.allclose(w.double().cpu(), wr, rtol=1e-4, atol=1e-5 * wr.abs().max().item())
        assert rel(V @ torch.diag_embed(w) @ V.transpose(1, 2), Z) < 1e-5


def test_ngd_native_eigh_matches_cpu(cuda, monkeypatch):
    """NGD with the native ragged eigh on the GPU tracks the fp64 CPU path as closely as
    NGD with fp32 LAPACK-style eigh (torch.linalg.eigh) does: the early-step Z matrices
    have degenerate eigenspaces, so any fp32 solver drifts by a few percent over 12 steps."""
    import torch.nn as nn
    import faster_distributed_training_amd.ops.eigh as E
    from faster_distributed_training_amd.optim.ngd import NGD
    from faster_distributed_training_amd.utils.flat import FlatParams

    def run(dev):
        torch.manual_seed(0)
        m = nn.Sequential(nn.Linear(40, 24, bias=False), nn.Linear(24, 10, bias=False)).to(dev)
        f = FlatParams(m)
        o = NGD(f, lr=0.05, momentum=0.9)
        for s in range(12):
            f.grad.copy_(torch.randn(f.numel, generator=torch.Generator().manual_seed(s)).to(dev))
            o.step()
        return f.data.cpu()

    ref = run("cpu")
    native = run(cuda)
    monkeypatch.setattr(E, "_use_native", lambda Z: False)
    lapack32 = run(cuda)
    e_nat, e_lap = rel(native, ref), rel(lapack32, ref)
    assert e_nat < max(2.0 * e_lap, 1e-3), (e_nat, e_lap)


def test_ngd_fused_small_math_matches_torch(cuda, monkeypatch):
    """The fused rank x rank update kernels (csrc/kernels/ngd.hip) vs the PyTorch formulation
    of the same NGD step, both against the fp64 CPU path over 14 steps: the early Z matrices
    have degenerate eigenspaces, so fp32 rounding differences rotate eigenvectors -- the
    fused path must drift no more than the PyTorch fp32 path does."""
    import torch.nn as nn
    import faster_distributed_training_amd.optim.ngd as N
    from faster_distributed_training_amd.utils.flat import FlatParams

    def run(dev, fused=True):
        monkeypatch.setattr(N, "FUSED", fused)
        torch.manual_seed(0)
        m = nn.Sequential(nn.Linear(40, 24), nn.Linear(24, 10, bias=False), nn.Linear(10, 7)).to(dev)
        f = FlatParams(m)
        o = N.NGD(f, lr=0.05, momentum=0.9, weight_decay=1e-4)
        for s in range(14):
            f.grad.copy_(torch.randn(f.numel, generator=torch.Generator().manual_seed(s)).to(dev))
            o.step()
        return f.data.cpu()

    ref = run("cpu")
    e_fused, e_torch = rel(run(cuda, True), ref), rel(run(cuda, False), ref)
    assert e_fused < max(2.0 * e_torch, 1e-3), (e_fused, e_torch)


@pytest.mark.parametrize("D,R,A,B", [(3, 2, 70, 3), (3, 2, 5000, 1), (5, 3, 33, 7), (8, 4, 1, 900)])
def test_ngd_small_proj_kernel_vs_torch(cuda, D, R, A, B):
    """ngd_small_proj (one streaming pass over a tiny-dim axis, canonical layout) against
    the GEMM formulation on the transposed copy: Xh, |X|^2, |Xh|^2, J = H^T X, H^T H."""
    from faster_distributed_training_amd.ops import _native
    nat = _native.native()
    torch.manual_seed(D * 100 + B)
    P = 3
    X = torch.randn(P, A, D, B, device=cuda)
    W = torch.randn(P, R, D, device=cuda) * 0.5
    buf = torch.zeros(2 * P + P * R * D + P * R * R, device=cuda)
    Y = torch.empty_like(X)
    J = buf[2 * P:2 * P + P * R * D]
    HH = buf[2 * P + P * R * D:]
    part = torch.full((nat.ngd_small_part_numel(P, A, D, B, R),), float("nan"), device=cuda)
    nat.ngd_small_proj(X.data_ptr(), Y.data_ptr(), W.data_ptr(), P, A, D, B, R, buf.data_ptr(), J.data_ptr(),
                       HH.data_ptr(), part.data_ptr(), _native.stream_ptr())
    Xt = X.double().transpose(2, 3).reshape(P, A * B, D)      # rows n = a * B + b
    Wd = W.double()
    H = torch.bmm(Xt, Wd.transpose(1, 2))
    Xh = Xt - torch.bmm(H, Wd)
    ref_Y = Xh.view(P, A, B, D).transpose(2, 3)
    torch.cuda.synchronize()
    assert rel(Y.double(), ref_Y) < 1e-5
    assert rel(buf[:P].double(), (Xt * Xt).sum((1, 2))) < 1e-5
    assert rel(buf[P:2 * P].double(), (Xh * Xh).sum((1, 2))) < 1e-5
    assert rel(J.view(P, R, D).double(), torch.bmm(H.transpose(1, 2), Xt)) < 1e-4
    assert rel(HH.view(P, R, R).double(), torch.bmm(H.transpose(1, 2), H)) < 1e-4
    # non-update form: only the two sums, J / HH untouched
    buf2 = torch.zeros(2 * P, device=cuda)
    Y2 = torch.empty_like(X)
    nat.ngd_small_proj(X.data_ptr(), Y2.data_ptr(), W.data_ptr(), P, A, D, B, R, buf2.data_ptr(), 0, 0,
                       part.data_ptr(), _native.stream_ptr())
    torch.cuda.synchronize()
    assert torch.equal(Y2, Y)
    assert torch.equal(buf2, buf[:2 * P])  # fixed-order partial sums: bitwise repeatable


@pytest.mark.parametrize("per", [4, 1000, 3 * 512 * 512 * 3])
def test_ngd_sumsq_rescale_vs_torch(cuda, per):
    """ngd_sumsq / ngd_rescale (float4 streaming, many workgroups per matrix) against the
    PyTorch expressions, including the NaN guard (matrix 1 falls back to X)."""
    from faster_distributed_training_amd.ops import _native
    nat = _native.native()
    G = 3
    X = torch.randn(G, per, device=cuda)
    Y = torch.randn(G, per, device=cuda)
    Y[1, per // 2] = float("nan")
    s = torch.zeros(2, G, device=cuda)
    sp = _native.stream_ptr()
    nat.ngd_sumsq(X.data_ptr(), per, G, s[0].data_ptr(), sp)
    nat.ngd_sumsq(Y.data_ptr(), per, G, s[1].data_ptr(), sp)
    ip, fp = (X.double() ** 2).sum(1), (Y.double() ** 2).sum(1)
    ref = torch.where(torch.isnan(fp).view(-1, 1), X.double(), Y.double() * torch.sqrt(ip / (fp + 1e-30)).view(-1, 1))
    nat.ngd_rescale(X.data_ptr(), Y.data_ptr(), per, G, s[0].data_ptr(), s[1].data_ptr(), sp)
    torch.cuda.synchronize()
    assert rel(s[0].double(), ip) < 1e-5
    assert torch.isnan(s[1, 1]) and rel(s[1, [0, 2]].double(), fp[[0, 2]]) < 1e-5
    assert torch.equal(Y[1], X[1])
    assert rel(Y.double(), ref) < 1e-5


def test_ngd_deferred_eigh_matches_sync(cuda, monkeypatch):
    """Update-step eigensolves deferred to one launch at the end of the optimizer step give
    the same trajectory as solving each axis level before the next (they only feed the
    next step's W); also counts the eigensolver launches of a steady update step."""
    import torch.nn as nn
    import faster_distributed_training_amd.optim.ngd as N
    import faster_distributed_training_amd.ops.eigh as E
    from faster_distributed_training_amd.utils.flat import FlatParams
    calls = []
    orig = E.eigh_many
    monkeypatch.setattr(E, "eigh_many", lambda Zs, *a, **k: calls.append(len(Zs)) or orig(Zs, *a, **k))

    def run(defer):
        monkeypatch.setattr(N, "DEFER", defer)
        torch.manual_seed(0)
        m = nn.Sequential(nn.Conv2d(4, 8, 3), nn.Conv2d(8, 8, 3), nn.Linear(8, 12)).to(cuda)
        f = FlatParams(m)
        o = N.NGD(f, lr=0.05, momentum=0.9, weight_decay=1e-4)
        for s in range(13):  # the last step (t = 12) is an update step
            calls.clear()
            f.grad.copy_(torch.randn(f.numel, generator=torch.Generator().manual_seed(s)).to(cuda))
            o.step()
        return f.data.clone(), list(calls)

    (a, ca), (b, cb) = run(True), run(False)
    assert ca == [sum(cb)], (ca, cb)  # one launch (all axes) vs one per axis level
    assert len(cb) > 1
    assert rel(a, b) < 1e-5


def test_ngd_small_axes_match_gemm_path(cuda, monkeypatch):
    """A conv model's NGD steps with the kh / kw axes on the streaming HIP pass vs the same
    axes on transpose + batched GEMMs, both against the fp64 CPU path over 14 steps."""
    import torch.nn as nn
    import faster_distributed_training_amd.optim.ngd as N
    from faster_distributed_training_amd.utils.flat import FlatParams
    used = []
    orig = N.NGState.small_ok

    def run(dev, small=True):
        monkeypatch.setattr(N.NGState, "small_ok",
                            (lambda self, G: orig(self, G) and not used.append(1)) if small else (lambda self, G: False))
        torch.manual_seed(0)
        m = nn.Sequential(nn.Conv2d(4, 6, 3), nn.Conv2d(6, 6, 3), nn.Conv2d(6, 5, 3, bias=False),
                          nn.Conv2d(5, 8, (1, 5))).to(dev)
        f = FlatParams(m)
        o = N.NGD(f, lr=0.05, momentum=0.9, weight_decay=1e-4)
        for s in range(14):
            f.grad.copy_(torch.randn(f.numel, generator=torch.Generator().manual_seed(s)).to(dev))
            o.step()
        return f.data.cpu()

    ref = run("cpu")
    e_small, e_gemm = rel(run(cuda, True), ref), rel(run(cuda, False), ref)
    assert used, "small-dim path not taken"
    assert e_small < max(2.0 * e_gemm, 1e-3), (e_small, e_gemm)


def test_ngd_pre_post_kernels_vs_torch(cuda):
    """ngd_pre_eigh / ngd_post_eigh against the PyTorch expressions of NGState._step."""
    from faster_distributed_training_amd.ops import _native
    nat = _native.native()
    torch.manual_seed(5)
    G, R, N, D, alpha, eta = 3, 7, 50.0, 20.0, 4.0, 0.1
    J = torch.randn(G, R, int(D), device=cuda)
    K = torch.bmm(J, J.transpose(1, 2))
    L = torch.randn(G, R, R, device=cuda)
    L = L + L.transpose(1, 2)
    d = torch.rand(G, R, device=cuda) + 0.1
    rho = torch.rand(G, device=cuda) + 0.05
    trXX = torch.rand(G, device=cuda) * 100 + 10
    # torch reference (ngd.py NGState._step)
    dsum = d.sum(dim=1)
    beta = rho * (1.0 + alpha) + alpha * dsum / D
    e = 1.0 / (beta.unsqueeze(1) / d + 1.0)
    ise = torch.rsqrt(e)
    zs = torch.clamp(torch.diagonal(K, dim1=1, dim2=2).sum(1), min=1.0)
    drho = d + rho.unsqueeze(1)
    c1, c2, c3 = ((eta / N) ** 2) / zs, ((eta / N) * (1.0 - eta)) / zs, ((1.0 - eta) ** 2) / zs
    oo = ise.unsqueeze(2) * ise.unsqueeze(1)
    o1 = ise.unsqueeze(2) * (ise * drho).unsqueeze(1)
    Zr = K * (c1.view(-1, 1, 1) * oo) + L * (c2.view(-1, 1, 1) * (o1 + o1.transpose(1, 2)))
    Zr = Zr + torch.diag_embed(c3.unsqueeze(1) * drho * drho)
    Z = torch.empty_like(Zr)
    ise_k, drho_k = torch.empty_like(d), torch.empty_like(d)
    zs_k, dsum_k = torch.empty_like(rho), torch.empty_like(rho)
    sp = _native.stream_ptr()
    nat.ngd_pre_eigh(K.data_ptr(), L.data_ptr(), d.data_ptr(), rho.data_ptr(), Z.data_ptr(), ise_k.data_ptr(),
                     drho_k.data_ptr(), zs_k.data_ptr(), dsum_k.data_ptr(), G, R, alpha, eta, N, D, sp)
    assert rel(Z, Zr) < 1e-5 and rel(ise_k, ise) < 1e-6 and rel(drho_k, drho) < 1e-6 and rel(zs_k, zs) < 1e-6
    c, U = torch.linalg.eigh(Zr.double())
    c, U = c.float().contiguous(), U.float().contiguous()
    cf, Uf = c.flip(1), U.flip(2)
    c_floor = ((rho * (1.0 - eta)) ** 2) / zs
    cf = torch.maximum(cf, c_floor.unsqueeze(1))
    sqc = torch.sqrt(cf) * torch.sqrt(zs).unsqueeze(1)
    rho1 = ((eta / N) * trXX + (1.0 - eta) * (D * rho + dsum) - sqc.sum(1)) / (D - R)
    floor = torch.clamp(1e-3 * 0.5 * sqc.max(dim=1).values, min=1e-10)
    d1 = torch.maximum(sqc - rho1.unsqueeze(1), floor.unsqueeze(1))
    rho1 = torch.maximum(rho1, floor)
    beta1 = rho1 * (1.0 + alpha) + alpha * d1.sum(1) / D
    e1 = 1.0 / (beta1.unsqueeze(1) / d1 + 1.0)
    wc = ((1.0 - eta) / (eta / N)) * drho
    lp = (eta / N) * torch.sqrt(e1) / sqc
    A = Uf.transpose(1, 2) * (lp.unsqueeze(2) * ise.unsqueeze(1))
    d_k, rho_k = d.clone(), rho.clone()
    # (not empty_like(A): A inherits the transposed strides of Uf.transpose(1, 2))
    A_k, wc_k = torch.empty(G, R, R, device=cuda), torch.empty_like(d)
    nat.ngd_post_eigh(c.data_ptr(), U.data_ptr(), ise_k.data_ptr(), drho_k.data_ptr(), zs_k.data_ptr(),
                      dsum_k.data_ptr(), trXX.data_ptr(), d_k.data_ptr(), rho_k.data_ptr(), A_k.data_ptr(),
                      wc_k.data_ptr(), G, R, alpha, eta, N, D, sp)
    torch.cuda.synchronize()
    assert rel(d_k, d1) < 1e-5, (d_k, d1)
    assert rel(rho_k, rho1) < 1e-5, (rho_k, rho1)
    assert rel(wc_k, wc) < 1e-6
    assert rel(A_k, A) < 1e-5


@pytest.mark.parametrize("D,R,A,B", [(9, 5, 40, 3), (64, 32, 1, 900), (512, 80, 300, 1), (40, 20, 7, 9),
                                     (2048, 80, 1, 100), (100, 50, 1, 1), (33, 17, 130, 1), (30522, 80, 1, 40),
                                     (500, 80, 9000, 1)])
def test_ngd_proj_kernel_vs_torch(cuda, D, R, A, B):
    """ngd_proj (fused H = X W^T, X - H W, sums, J, H^T H in the parameter's own layout)
    against the fp64 GEMM formulation on the transposed copy."""
    from faster_distributed_training_amd.ops import _native
    nat = _native.native()
    torch.manual_seed(D * 7 + B)
    P = 3
    X = torch.randn(P, A, D, B, device=cuda)
    W = torch.randn(P, R, D, device=cuda) / D ** 0.5
    ip, fp = torch.zeros(P, device=cuda), torch.zeros(P, device=cuda)
    J = torch.zeros(P, R, D, device=cuda)
    HH = torch.zeros(P, R, R, device=cuda)
    Y = torch.empty_like(X)
    Hb = torch.full((nat.ngd_proj_hbuf_numel(P, A, D, B, R, True, True, True),), float("nan"), device=cuda)
    sp = _native.stream_ptr()
    nat.ngd_proj(X.data_ptr(), Y.data_ptr(), W.data_ptr(), Hb.data_ptr(), P, A, D, B, R, ip.data_ptr(),
                 fp.data_ptr(), J.data_ptr(), HH.data_ptr(), sp)
    Xt = X.double().transpose(2, 3).reshape(P, A * B, D)      # rows n = a * B + b
    Wd = W.double()
    H = torch.bmm(Xt, Wd.transpose(1, 2))
    Xh = Xt - torch.bmm(H, Wd)
    ref_Y = Xh.view(P, A, B, D).transpose(2, 3)
    torch.cuda.synchronize()
    assert rel(Y.double(), ref_Y) < 1e-5
    assert rel(ip.double(), (Xt * Xt).sum((1, 2))) < 1e-5
    assert rel(fp.double(), (Xh * Xh).sum((1, 2))) < 1e-5
    assert rel(J.double(), torch.bmm(H.transpose(1, 2), Xt)) < 1e-4
    assert rel(HH.double(), torch.bmm(H.transpose(1, 2), H)) < 1e-4
    # non-update form with |X|^2 supplied: only |Y|^2, no J / H^T H
    fp2 = torch.zeros(P, device=cuda)
    Y2 = torch.empty_like(X)
    nat.ngd_proj(X.data_ptr(), Y2.data_ptr(), W.data_ptr(), Hb.data_ptr(), P, A, D, B, R, 0, fp2.data_ptr(), 0, 0,
                 sp)
    torch.cuda.synchronize()
    assert torch.equal(Y2, Y)  # every cross-workgroup sum is a fixed-order slab sum: bitwise repeatable
    assert torch.equal(fp2, fp)
    # and a second full (update-form) call reproduces ip, fp, J, H^T H exactly
    ip3, fp3 = torch.zeros(P, device=cuda), torch.zeros(P, device=cuda)
    J3, HH3 = torch.zeros_like(J), torch.zeros_like(HH)
    Y3 = torch.empty_like(X)
    nat.ngd_proj(X.data_ptr(), Y3.data_ptr(), W.data_ptr(), Hb.data_ptr(), P, A, D, B, R, ip3.data_ptr(),
                 fp3.data_ptr(), J3.data_ptr(), HH3.data_ptr(), sp)
    torch.cuda.synchronize()
    assert torch.equal(Y3, Y) and torch.equal(ip3, ip) and torch.equal(fp3, fp)
    assert torch.equal(J3, J) and torch.equal(HH3, HH)
    # the matrix-core form (default) against the VALU form: the same k-ordered fp32 fmaf
    # chains (v_mfma_f32_16x16x4_f32 rounds once per product, in k order) -> identical bits
    prev = nat.ngd_mfma(0)
    try:
        ip4, fp4 = torch.zeros(P, device=cuda), torch.zeros(P, device=cuda)
        J4, HH4 = torch.zeros_like(J), torch.zeros_like(HH)
        Y4 = torch.empty_like(X)
        nat.ngd_proj(X.data_ptr(), Y4.data_ptr(), W.data_ptr(), Hb.data_ptr(), P, A, D, B, R, ip4.data_ptr(),
                     fp4.data_ptr(), J4.data_ptr(), HH4.data_ptr(), sp)
        torch.cuda.synchronize()
    finally:
        nat.ngd_mfma(prev)
    assert prev == 1
    assert torch.equal(Y4, Y), rel(Y4.double(), Y.double())
    assert torch.equal(J4, J), rel(J4.double(), J.double())
    assert torch.equal(ip4, ip) and torch.equal(HH4, HH)
    # |Y|^2: the same Y, but each thread's partial sum covers other elements (C-fragment map)
    assert rel(fp4.double(), fp.double()) < 1e-6


def test_ngd_proj_axes_match_gemm_path(cuda, monkeypatch):
    """Linear + conv model NGD steps with every dim >= 9 axis on the fused projection kernel
    vs the transpose + batched-GEMM path, both against the fp64 CPU path over 14 steps
    (update and non-update steps, the initialisation iterations included)."""
    import torch.nn as nn
    import faster_distributed_training_amd.optim.ngd as N
    from faster_distributed_training_amd.utils.flat import FlatParams
    used = []
    orig = N.NGState.proj_ok

    def run(dev, proj=True):
        monkeypatch.setattr(N.NGState, "proj_ok",
                            (lambda self, G: orig(self, G) and not used.append(1)) if proj else (lambda self, G: False))
        torch.manual_seed(0)
        m = nn.Sequential(nn.Conv2d(12, 20, 3), nn.Conv2d(20, 16, 1), nn.Linear(16, 200), nn.Linear(200, 12),
                          nn.BatchNorm1d(12)).to(dev)
        f = FlatParams(m)
        o = N.NGD(f, lr=0.05, momentum=0.9, weight_decay=1e-4)
        for s in range(14):
            f.grad.copy_(torch.randn(f.numel, generator=torch.Generator().manual_seed(s)).to(dev))
            o.step()
        return f.data.cpu()

    ref = run("cpu")
    e_proj, e_gemm = rel(run(cuda, True), ref), rel(run(cuda, False), ref)
    assert used, "fused projection path not taken"
    assert e_proj < max(2.0 * e_gemm, 1e-3), (e_proj, e_gemm)



def test_ngd_side_stream_eigh_matches_inline(cuda, monkeypatch):
    """The deferred eigensolve + state update on a side stream (overlapping the caller's
    next work, here a matmul chain queued right after every step) gives bitwise the same
    trajectory and preconditioner state as solving it inline on the caller's stream, over
    the initialisation schedule and several update periods (the preconditioning path has
    no order-dependent atomics, test_ngd_step_bitwise_repeatable)."""
    import torch.nn as nn
    import faster_distributed_training_amd.optim.ngd as N
    from faster_distributed_training_amd.utils.flat import FlatParams

    def run(overlap):
        torch.manual_seed(0)
        m = nn.Sequential(nn.Conv2d(12, 20, 3), nn.Conv2d(20, 16, 1), nn.Linear(16, 200), nn.Linear(200, 12)).to(cuda)
        f = FlatParams(m)
        o = N.NGD(f, lr=0.05, momentum=0.9, weight_decay=1e-4, overlap_eigh=overlap)
        busy = torch.randn(2048, 2048, device=cuda)
        used = 0
        for s in range(18):
            f.grad.copy_(torch.randn(f.numel, generator=torch.Generator().manual_seed(s)).to(cuda))
            o.step()
            used += o._pending is not None
            busy = busy @ busy / 2048.0  # the caller's next work, concurrent with the side stream
        return f.data.clone(), [(st.W.clone(), st.d.clone(), st.rho.clone()) for st in o._states()], used

    (a, sa, used), (b, sb, _) = run(True), run(False)
    assert used >= 6  # every update step deferred its solve to the side stream
    assert torch.equal(a, b)
    for x, y in zip(sa, sb):
        assert all(torch.equal(u, v) for u, v in zip(x, y))


def test_ngd_step_bitwise_repeatable(cuda):
    """Two identical NGD runs (general-axis projection, kh / kw streaming axes, 1-D
    parameters, eigensolves, side-stream state updates) give bitwise identical parameters:
    no cross-workgroup atomics in the preconditioning path."""
    import torch.nn as nn
    import faster_distributed_training_amd.optim.ngd as N
    from faster_distributed_training_amd.utils.flat import FlatParams

    def run():
        torch.manual_seed(0)
        m = nn.Sequential(nn.Conv2d(12, 20, 3), nn.Conv2d(20, 16, 1), nn.Linear(16, 200), nn.Linear(200, 12),
                          nn.BatchNorm1d(12)).to(cuda)
        f = FlatParams(m)
        o = N.NGD(f, lr=0.05, momentum=0.9, weight_decay=1e-4)
        for s in range(14):
            f.grad.copy_(torch.randn(f.numel, generator=torch.Generator().manual_seed(s)).to(cuda))
            o.step()
        return f.data.clone()

    assert torch.equal(run(), run())



# ---------------------------------------------------------------- NGD R x R products
@pytest.mark.parametrize("G,R,D", [(3, 1, 9), (2, 17, 27), (4, 32, 64), (3, 80, 513), (2, 80, 4608), (1, 128, 300)])
def test_ngd_gram_and_wupdate_match_fp64(cuda, G, R, D):
    """ngd_gram (K = J J^T, L = J W^T: split-d partial tiles summed in a fixed order) and
    ngd_wupdate (W <- A (J + wc W) in place) against fp64 products; repeated calls are
    bitwise identical."""
    from faster_distributed_training_amd.optim.ngd import gram, w_update
    g = torch.Generator(device=cuda).manual_seed(G * 1000 + R * 10 + D)
    J = torch.randn(G, R, D, device=cuda, generator=g)
    W = torch.randn(G, R, D, device=cuda, generator=g)
    K, L = gram(J, W)
    Jd, Wd = J.double(), W.double()
    assert rel(K, Jd @ Jd.transpose(1, 2)) < 1e-6 and rel(L, Jd @ Wd.transpose(1, 2)) < 1e-6
    assert torch.equal(K, K.transpose(1, 2))  # symmetric by construction
    K2, L2 = gram(J, W)
    assert torch.equal(K, K2) and torch.equal(L, L2)
    K3, L3 = gram(J)
    assert L3 is None and torch.equal(K3, K)
    A = torch.randn(G, R, R, device=cuda, generator=g)
    wc = torch.rand(G, R, device=cuda, generator=g)
    want = A.double() @ (Jd + wc.double().unsqueeze(2) * Wd)
    Wn = W.clone()
    w_update(A, J, wc, Wn)
    assert rel(Wn, want) < 1e-6
