"""Flat fused optimizers (CPU path = the kernel oracle) against torch.optim / reference
update rules, and the batched NGD against the reference OnlineNaturalGradient."""
import math

import pytest
import torch
import torch.nn as nn

from faster_distributed_training_amd.optim import flat_optim as O
from faster_distributed_training_amd.optim.ngd import NGD, NGState, OnlineNaturalGradient, default_rank
from faster_distributed_training_amd.utils.flat import FlatParams

from reference_oracle import load


def _net(seed=0):
    torch.manual_seed(seed)
    return nn.Sequential(nn.Linear(6, 5), nn.Tanh(), nn.Linear(5, 3))


def _grads(m, seed):
    g = torch.Generator().manual_seed(seed)
    return [torch.randn(p.shape, generator=g) for p in m.parameters()]


def _run(flat_opt_ctor, torch_opt_ctor, steps=5):
    a, b = _net(), _net()
    flat = FlatParams(a)
    oa = flat_opt_ctor(flat)
    ob = torch_opt_ctor(b.parameters())
    for s in range(steps):
        for p, g in zip(a.parameters(), _grads(a, s)):
            p.grad.copy_(g)
        for p, g in zip(b.parameters(), _grads(b, s)):
            p.grad = g.clone()
        oa.step()
        ob.step()
    for pa, pb in zip(a.parameters(), b.parameters()):
        assert torch.allclose(pa, pb, atol=1e-6, rtol=1e-5)


@pytest.mark.parametrize("mom,nest,damp,wd", [(0.0, False, 0.0, 0.0), (0.9, False, 0.0, 5e-4), (0.9, True, 0.0, 1e-4),
                                              (0.9, False, 0.1, 0.0)])
def test_sgd_matches_torch(mom, nest, damp, wd):
    _run(lambda f: O.SGD(f, lr=0.1, momentum=mom, nesterov=nest, dampening=damp, weight_decay=wd),
         lambda ps: torch.optim.SGD(ps, lr=0.1, momentum=mom, nesterov=nest, dampening=damp, weight_decay=wd))


@pytest.mark.parametrize("adamw", [False, True])
def test_adam_matches_torch(adamw):
    ctor = torch.optim.AdamW if adamw else torch.optim.Adam
    _run(lambda f: O.Adam(f, lr=1e-2, weight_decay=1e-2, adamw=adamw), lambda ps: ctor(ps, lr=1e-2, weight_decay=1e-2))


def _madgrad_reference(params, grads_per_step, lr, momentum, wd, eps=1e-6):
    """Textbook MADGRAD (Defazio & Jelassi 2021, Alg. 1) with the public implementation's
    conventions: weight decay added to the gradient and the step size lr + eps."""
    ps = [p.clone() for p in params]
    x0 = [p.clone() for p in ps]
    s = [torch.zeros_like(p) for p in ps]
    nu = [torch.zeros_like(p) for p in ps]
    for k, grads in enumerate(grads_per_step):
        ck = 1 - momentum
        lamb = (lr + eps) * math.sqrt(k + 1)
        for i, (p, g) in enumerate(zip(ps, grads)):
            g = g + wd * p if wd else g
            s[i] += lamb * g
            nu[i] += lamb * g * g
            rms = nu[i].pow(1 / 3) + eps
            z = x0[i] - s[i] / rms
            ps[i] = (1 - ck) * p + ck * z
    return ps


def test_madgrad_matches_paper_rule():
    a = _net()
    flat = FlatParams(a)
    init = [p.detach().clone() for p in a.parameters()]
    opt = O.MADGRAD(flat, lr=1e-2, momentum=0.9, weight_decay=1e-4)
    steps = [_grads(a, s) for s in range(4)]
    for gs in steps:
        for p, g in zip(a.parameters(), gs):
            p.grad.copy_(g)
        opt.step()
    ref = _madgrad_reference(init, steps, 1e-2, 0.9, 1e-4)
    for p, r in zip(a.parameters(), ref):
        assert torch.allclose(p, r, atol=1e-6, rtol=1e-5)


def test_mirror_madgrad_runs_and_descends():
    torch.manual_seed(0)
    w = nn.Linear(4, 1)
    flat = FlatParams(w)
    opt = O.MirrorMADGRAD(flat, lr=0.05, momentum=0.9)
    x = torch.randn(64, 4)
    y = x @ torch.tensor([[1.0], [-2.0], [0.5], [3.0]])
    losses = []
    for _ in range(60):
        loss = ((w(x) - y) ** 2).mean()
        loss.backward()
        opt.step()
        losses.append(loss.item())
    assert losses[-1] < 0.2 * losses[0]


def test_grad_clipper_and_scaled_step():
    a, b = _net(), _net()
    fa = FlatParams(a)
    clip = O.GradClipper(fa)
    oa = O.SGD(fa, lr=0.1)
    ob = torch.optim.SGD(b.parameters(), lr=0.1)
    gs = [g * 50 for g in _grads(a, 3)]
    for p, g in zip(a.parameters(), gs):
        p.grad.copy_(g)
    for p, g in zip(b.parameters(), gs):
        p.grad = g.clone()
    clip(1.0)
    oa.step(grad_scale=clip.coef)
    nb = torch.nn.utils.clip_grad_norm_(b.parameters(), 1.0)
    ob.step()
    assert abs(float(clip.norm) - float(nb)) < 1e-4 * float(nb)
    for pa, pb in zip(a.parameters(), b.parameters()):
        assert torch.allclose(pa, pb, atol=1e-6)


def test_lr_scheduler_drives_flat_optimizer():
    a = _net()
    opt = O.SGD(FlatParams(a), lr=1.0)
    sch = torch.optim.lr_scheduler.MultiStepLR(opt, [2, 4], gamma=0.2)
    lrs = []
    for _ in range(5):
        lrs.append(opt.group["lr"])
        sch.step()
    assert lrs == pytest.approx([1.0, 1.0, 0.2, 0.2, 0.04])


def test_optimizer_state_dict_roundtrip():
    a = _net()
    flat = FlatParams(a)
    opt = O.MADGRAD(flat, lr=1e-2)
    for s in range(2):
        for p, g in zip(a.parameters(), _grads(a, s)):
            p.grad.copy_(g)
        opt.step()
    sd = opt.state_dict()
    b = _net()
    fb = FlatParams(b)
    with torch.no_grad():
        fb.data.copy_(flat.data)
    ob = O.MADGRAD(fb, lr=1e-2)
    ob.load_state_dict(sd)
    assert ob.k == opt.k
    for p, g in zip(a.parameters(), _grads(a, 9)):
        p.grad.copy_(g)
    for p, g in zip(b.parameters(), _grads(b, 9)):
        p.grad.copy_(g)
    opt.step()
    ob.step()
    assert torch.allclose(flat.data, fb.data, atol=1e-7)


# ---------------------------------------------------------------- NGD
def test_default_rank():
    assert default_rank(2) == 1 and default_rank(64) == 32 and default_rank(2048) == 80 and default_rank(5) == 3


@pytest.mark.parametrize("shape,axis", [((12, 7), 0), ((12, 7), 1), ((6, 5, 3), 1), ((40,), 0)])
def test_online_natural_gradient_matches_reference(shape, axis):
    """20 steps (init, every-step updates for t < 10, then update_period 4) in fp64.

    A 1-D parameter gives N = 1 row per step: the R x R matrix Z then has a large
    degenerate eigenspace, whose basis LAPACK picks arbitrarily, so the two
    implementations agree exactly only on the first step and within a few percent
    afterwards (both preserve the gradient norm exactly)."""
    ref = load("ngd_optimizer")
    torch.manual_seed(0)
    p = torch.zeros(shape, dtype=torch.float64)
    ra = ref.OnlineNaturalGradient(p, axis, alpha=4.0, update_period=4, eta=0.1)
    oa = OnlineNaturalGradient(p, axis, alpha=4.0, update_period=4, eta=0.1)
    degenerate = len(shape) == 1
    for step in range(20):
        g = torch.randn(shape, dtype=torch.float64) * (1 + step % 3)
        a = oa.precondition_directions(g.clone())
        b = ra.precondition_directions(g.clone())
        assert torch.allclose(a.norm(), g.norm()) and torch.allclose(b.norm(), g.norm())
        err = ((a - b).norm() / b.norm()).item()
        assert err < (1e-5 if step == 0 else 0.1) if degenerate else err < 1e-10, (step, err)


def test_ngd_optimizer_matches_reference():
    """Full optimizer (weight decay -> per-axis preconditioning -> momentum) vs the
    reference NGD.  Bias-free layers: 1-D parameters are the degenerate N = 1 case (see
    above) where fp32 (flat buffer) vs fp64 rounding already selects different bases."""
    ref = load("ngd_optimizer")
    torch.manual_seed(0)
    ma = nn.Sequential(nn.Linear(8, 6, bias=False), nn.Linear(6, 3, bias=False)).double()
    mb = nn.Sequential(nn.Linear(8, 6, bias=False), nn.Linear(6, 3, bias=False)).double()
    mb.load_state_dict(ma.state_dict())
    flat = FlatParams(ma)  # fp32 flat buffer: compare with fp32 tolerance
    oa = NGD(flat, lr=0.05, momentum=0.9, weight_decay=1e-4)
    ob = ref.NGD(mb.parameters(), lr=0.05, momentum=0.9, weight_decay=1e-4)
    for s in range(12):
        g = torch.Generator().manual_seed(100 + s)
        gs = [torch.randn(p.shape, generator=g, dtype=torch.float64) for p in mb.parameters()]
        for p, gg in zip(ma.parameters(), gs):
            p.grad.copy_(gg)
        for p, gg in zip(mb.parameters(), gs):
            p.grad = gg.clone()
        oa.step()
        ob.step()
    for pa, pb in zip(ma.parameters(), mb.parameters()):
        assert torch.allclose(pa.double(), pb, rtol=1e-4, atol=1e-5)


def test_ngd_batched_groups_equal_per_tensor():
    """Batching same-shape parameters into one NGState equals running them separately."""
    torch.manual_seed(0)
    G, N, D = 3, 10, 6
    st = NGState(G, D, default_rank(D), 4.0, 4, 0.1, torch.float64, "cpu")
    singles = [NGState(1, D, default_rank(D), 4.0, 4, 0.1, torch.float64, "cpu") for _ in range(G)]
    for _ in range(8):
        X = torch.randn(G, N, D, dtype=torch.float64)
        out = st.precondition(X.clone())
        for i in range(G):
            assert torch.allclose(out[i], singles[i].precondition(X[i:i + 1].clone())[0], atol=1e-10)


def test_ngd_balanced_partition_resnet50():
    """ZeRO-2 NGD sharding by preconditioning cost (utils/flat.ngd_balanced_order): every
    parameter in exactly one run, no run above 1.15x the even element share, and the
    per-rank NGD cost spread far tighter than the element-balanced contiguous split."""
    from faster_distributed_training_amd.models.resnet import resnet50
    from faster_distributed_training_amd.utils.flat import FlatParams, ngd_cost
    m = resnet50(10)
    spread = {}
    for bal in ("numel", "ngd"):
        f = FlatParams(m, partition=8, balance=bal)
        assert sorted(id(s.param) for s in f.slots) == sorted(id(p) for p in m.parameters())
        costs = [sum(ngd_cost(tuple(s.shape)) for s in f.slots[a:b]) for a, b in f.runs]
        spread[bal] = max(costs) / (sum(costs) / len(costs))
        if bal == "ngd":
            total = sum(p.numel() for p in m.parameters())
            assert f.chunk <= 1.15 * total / 8 + 4096
    assert spread["ngd"] < 1.1 and spread["ngd"] < spread["numel"], spread


def test_ngd_shape_groups_as_flat_views_equal_stacked(monkeypatch):
    """A model that asks for same-shape parameters to sit back to back in the flat buffers
    (``flat_adjacent``, the Transformer does) gets its NGD shape groups as VIEWS of the flat
    gradient (no stack / scatter copies, optim/ngd.py ``_group_view``) -- the same steps as
    with stacked copies, and the fused Q/K/V projection reads its weights as one view."""
    import faster_distributed_training_amd.optim.ngd as N
    from faster_distributed_training_amd.models.transformer import Transformer
    from faster_distributed_training_amd.ops.linear import stacked

    def run(views):
        torch.manual_seed(0)
        m = Transformer(4, 300, n_layers=2, d_model=64, h=4, d_ff=128, d_hidden=128, maxlen=64).double()
        f = FlatParams(m, dtype=torch.float64)
        if not views:
            monkeypatch.setattr(N, "_group_view", lambda grad, slots: None)
        o = NGD(f, lr=0.05, momentum=0.9, weight_decay=1e-4)
        g = torch.Generator().manual_seed(1)
        for _ in range(12):
            f.grad.copy_(torch.randn(f.numel, generator=g, dtype=torch.float64))
            o.step()
        monkeypatch.undo()
        return f, m

    fv, m = run(True)
    fs, _ = run(False)
    assert torch.equal(fv.data, fs.data)
    o = NGD(fv, lr=0.05)
    o._build_groups()
    assert sum(N._group_view(fv.grad, slots) is not None for sg, slots in o.groups if sg.axes) >= 3
    heads = m.sublayer_attention[0].multiheads.heads
    w = stacked([l.weight for l in heads])
    assert w.data_ptr() == heads[0].weight.data_ptr() and w.shape == (192, 64)
    assert torch.equal(w, torch.cat([l.weight for l in heads]))


def test_ngd_plain_steps_defer_clip_scale_to_sgd(monkeypatch):
    """On a plain (non-update) NGD step the preconditioning is homogeneous of degree one in the
    gradient, so the clip coefficient applied by the final SGD kernel equals scaling the
    gradient first (NGD._scale_deferrable): same parameters to fp64 rounding over the 10-step
    initialisation schedule plus 3 update periods."""
    import faster_distributed_training_amd.optim.ngd as N

    def run(defer):
        monkeypatch.setattr(N, "DEFER_SCALE", defer)
        torch.manual_seed(0)
        m = nn.Sequential(nn.Linear(40, 24), nn.Linear(24, 10)).double()
        f = FlatParams(m, dtype=torch.float64)
        o = NGD(f, lr=0.05, momentum=0.9)
        g = torch.Generator().manual_seed(1)
        scale = torch.tensor([0.37], dtype=torch.float64)
        for _ in range(22):
            f.grad.copy_(torch.randn(f.numel, generator=g, dtype=torch.float64))
            o.step(grad_scale=scale)
        return f.data.clone()

    a, b = run(True), run(False)
    assert ((a - b).norm() / b.norm()).item() < 1e-10


def test_flat_optimizer_state_follows_parameter_order():
    """Flat optimizer state (momentum / second moments as flat vectors) is saved with its slot
    table (name, offset, numel): loaded into another slot order of the same parameters (a
    model's ``flat_adjacent`` groups, a reversed layout) it is moved slot by slot onto the
    right parameters.  A dict with only the layout fingerprint loads into that exact layout
    only, and one with neither (written before both existed) is refused -- the element count
    alone cannot tell a reordered buffer from the same one."""
    torch.manual_seed(0)
    m = nn.Sequential(nn.Linear(8, 8), nn.Linear(8, 6))
    a = O.MADGRAD(FlatParams(m, reverse=True), lr=1e-3)
    a.flat.grad.normal_()
    a.step()
    sd = a.state_dict()
    fb = FlatParams(nn.Sequential(nn.Linear(8, 8), nn.Linear(8, 6)), reverse=False)
    b = O.MADGRAD(fb, lr=1e-3)
    b.load_state_dict(sd)
    sa, sb = a.state["__flat__"], b.state["__flat__"]
    moved = 0
    for k, v in sa.items():
        if torch.is_tensor(v) and v.dim() == 1 and v.numel() == a.flat.numel:
            for sl in a.flat.slots:
                dst = next(t for t in fb.slots if t.name == sl.name)
                assert torch.equal(sb[k][dst.offset:dst.offset + dst.numel], v[sl.offset:sl.offset + sl.numel])
            moved += 1
    assert moved >= 2
    legacy = {k: v for k, v in sd.items() if k not in ("slots",)}
    with pytest.raises(ValueError, match="parameter order"):
        O.MADGRAD(FlatParams(nn.Sequential(nn.Linear(8, 8), nn.Linear(8, 6)), reverse=False), lr=1e-3).load_state_dict(legacy)
    O.MADGRAD(FlatParams(nn.Sequential(nn.Linear(8, 8), nn.Linear(8, 6)), reverse=True), lr=1e-3).load_state_dict(legacy)
    older = {k: v for k, v in sd.items() if k not in ("slots", "layout")}
    with pytest.raises(ValueError, match="cannot be verified"):
        O.MADGRAD(FlatParams(nn.Sequential(nn.Linear(8, 8), nn.Linear(8, 6)), reverse=True), lr=1e-3).load_state_dict(older)
    other = O.MADGRAD(FlatParams(nn.Sequential(nn.Linear(8, 8), nn.Linear(8, 7)), reverse=True), lr=1e-3)
    with pytest.raises(ValueError):
        other.load_state_dict(sd)
