"""The optimizer's fused update-and-pack step (csrc/kernels/optim_pack.hip): SGD / MADGRAD
update the flat buffer AND write the convolutions' packed bf16 layouts in one launch, so the
engine's forward skips its repack pass.  Oracle: the plain flat step followed by the standalone
repack (pack_weights) -- the two must agree bitwise (same update math, same bf16 rounding)."""
import copy
from types import SimpleNamespace

import pytest
import torch
import torch.nn as nn
import torch.nn.functional as F


class _Net(nn.Module):
    """Every conv layout the engine packs: a 3-channel stem (Cxp 8 padding, forward layout
    only), 3x3 / 1x1 / 2x2 kernels, plus non-conv parameters between them."""

    def __init__(self):
        super().__init__()
        self.stem = nn.Conv2d(3, 64, 3, padding=1, bias=False)
        self.bn = nn.BatchNorm2d(64)
        self.c3 = nn.Conv2d(64, 64, 3, padding=1, bias=False)
        self.c1 = nn.Conv2d(64, 256, 1, bias=False)
        self.c2 = nn.Conv2d(256, 128, 2, stride=2, bias=False)
        self.fc = nn.Linear(128, 10)


class _FakePlan:
    """The Plan surface the optimizer uses, over hand-made units."""

    def __init__(self, net, dev):
        from faster_distributed_training_amd.ops import conv_igemm as ci
        from faster_distributed_training_amd.ops.resnet_fused import Plan
        self.fsdp = None
        self.units = []
        for conv in (net.stem, net.c3, net.c1, net.c2):
            co, cin, k, _ = conv.weight.shape
            shp = ci.ConvShape(cin, co, k, conv.stride[0], conv.padding[0])
            wf, wd = ci.alloc_packed(shp, dev, dgrad=cin >= 8)
            self.units.append(SimpleNamespace(w=conv.weight, shp=shp, wf=wf, wd=wd))
        for name in ("update_table", "mark_opt_packed", "invalidate_pack", "pack_fresh", "_weights_version"):
            setattr(self, name, getattr(Plan, name).__get__(self))

    def repack(self):
        from faster_distributed_training_amd.ops import conv_igemm as ci
        ci.pack_weights([(u.w.detach(), u.wf, u.wd, u.shp) for u in self.units])


@pytest.fixture(autouse=True)
def _pack_in_opt(monkeypatch):
    from faster_distributed_training_amd.ops import resnet_fused
    monkeypatch.setattr(resnet_fused, "PACK_IN_OPT", True)


def _setup(cuda, opt_name, seed=0):
    from faster_distributed_training_amd.optim.flat_optim import MADGRAD, SGD
    from faster_distributed_training_amd.utils.flat import FlatParams
    torch.manual_seed(seed)
    net = _Net()
    out = []
    for fused in (False, True):
        m = copy.deepcopy(net).to(cuda)
        flat = FlatParams(m, device=cuda)
        plan = _FakePlan(m, cuda)
        plan.repack()
        if fused:
            flat.pack_owner = SimpleNamespace(_plan=plan)
        if opt_name == "madgrad":
            opt = MADGRAD(flat, lr=1e-2, momentum=0.9, weight_decay=1e-4)
        elif opt_name == "madgrad0":
            opt = MADGRAD(flat, lr=1e-2, momentum=0.0, weight_decay=1e-4, decouple_decay=True)
        else:
            opt = SGD(flat, lr=0.05, momentum=0.9, weight_decay=5e-4, nesterov=True)
        out.append((m, flat, plan, opt))
    return out


def _same(a, b):
    return a.shape == b.shape and torch.equal(a.view(torch.int16) if a.dtype == torch.bfloat16 else a,
                                              b.view(torch.int16) if b.dtype == torch.bfloat16 else b)


@pytest.mark.gpu
@pytest.mark.parametrize("opt_name", ["madgrad", "madgrad0", "sgd"])
def test_fused_update_pack_equals_step_then_repack(cuda, opt_name):
    (ma, fa, pa, oa), (mb, fb, pb, ob) = _setup(cuda, opt_name)
    g = torch.Generator(device=cuda).manual_seed(1)
    scale = torch.tensor([0.7], device=cuda)
    for step in range(3):
        grad = torch.randn(fa.numel, device=cuda, generator=g) * 0.1
        fa.grad.copy_(grad)
        fb.grad.copy_(grad)
        oa.step(grad_scale=scale if step == 1 else None)
        pa.repack()
        ob.step(grad_scale=scale if step == 1 else None)
        torch.cuda.synchronize()
        assert ob._packed and pb.pack_fresh()
        assert _same(fa.data, fb.data), f"weights differ after step {step}"
        for k, v in oa.state["__flat__"].items():
            if torch.is_tensor(v):
                assert _same(v, ob.state["__flat__"][k]), k
        assert not fb.grad.any()
        for ua, ub in zip(pa.units, pb.units):
            assert _same(ua.wf, ub.wf), ("forward layout", tuple(ua.w.shape))
            if ua.wd is not None:
                assert _same(ua.wd, ub.wd), ("dgrad layout", tuple(ua.w.shape))
    # a torch write to a weight (e.g. load_state_dict) ends the claim
    with torch.no_grad():
        mb.c3.weight.mul_(1.0)
    assert not pb.pack_fresh()


@pytest.mark.gpu
def test_fused_update_pack_skipped_step_keeps_layouts(cuda):
    (_, _, _, _), (mb, fb, pb, ob) = _setup(cuda, "madgrad")
    fb.grad.normal_()
    w0, wf0 = fb.data.clone(), [u.wf.clone() for u in pb.units]
    found = torch.ones(1, device=cuda, dtype=torch.int32)
    ob.step(found_inf=found)
    torch.cuda.synchronize()
    assert torch.equal(fb.data, w0) and not fb.grad.any()
    assert int(ob.kskip.item()) == 1
    assert all(_same(u.wf, w) for u, w in zip(pb.units, wf0))
    assert pb.pack_fresh()  # unchanged weights: the layouts still match them


@pytest.mark.gpu
def test_engine_training_with_optimizer_packed_weights(cuda):
    """ResNet-50 through the engine with HIP graphs, deterministic kernels: weights trained with
    the optimizer writing the packed layouts (forward graph captured without its repack) equal
    the ones trained with the per-forward repack, step for step; a checkpoint load between steps
    is picked up (the replay repacks)."""
    from faster_distributed_training_amd.models import resnet as R
    from faster_distributed_training_amd.ops import _native
    from faster_distributed_training_amd.optim.flat_optim import MADGRAD
    from faster_distributed_training_amd.utils.flat import FlatParams
    _native.set_deterministic(True)
    try:
        torch.manual_seed(0)
        base = R.resnet50(10).to(cuda)
        runs = []
        for fused in (False, True):
            m = copy.deepcopy(base)
            m.fast_path = True
            m.graph_engine = True
            flat = FlatParams(m, device=cuda)
            if fused:
                flat.pack_owner = m
            runs.append((m, flat, MADGRAD(flat, lr=1e-3, momentum=0.9, weight_decay=1e-4)))
        g = torch.Generator().manual_seed(3)
        x = torch.randn(64, 3, 32, 32, generator=g).to(cuda)
        y = torch.randint(0, 10, (64,), generator=g).to(cuda)
        sd_mid = None
        for step in range(6):
            if step == 4:  # out-of-band weight write between replays
                sd_mid = {k: v.clone() for k, v in runs[0][0].state_dict().items()}
                for v in sd_mid.values():
                    if v.dim() == 4:  # every conv weight
                        v.mul_(0.5)
                for m, _, _ in runs:
                    m.load_state_dict(sd_mid)
            losses = []
            for m, flat, opt in runs:
                with torch.autocast("cuda", dtype=torch.bfloat16):
                    out = m(x)
                loss = F.cross_entropy(out.float(), y)
                loss.backward()
                opt.step()
                losses.append(loss.detach())
            torch.cuda.synchronize()
            assert torch.equal(losses[0], losses[1]), (step, losses)
            assert torch.equal(runs[0][1].data, runs[1][1].data), f"weights differ after step {step}"
        plan = runs[1][0]._plan
        st = list(plan._graphs.values())[0]
        assert st.stage == "ready" and not st.repacks  # captured without the repack pass
        assert runs[1][2]._packed and plan.pack_fresh()
        assert sd_mid is not None
    finally:
        _native.set_deterministic(False)


def test_out_of_band_writes_drop_the_packed_claim():
    from faster_distributed_training_amd.utils.flat import FlatParams
    net = _Net()
    flat = FlatParams(net)
    plan = SimpleNamespace(_pk=("x", 1))
    plan.invalidate_pack = lambda: plan.__dict__.pop("_pk", None)
    flat.pack_owner = SimpleNamespace(_plan=plan)
    flat.refresh_shadow()  # (DDP's initial broadcast, a checkpoint restore, load_from_params)
    assert "_pk" not in plan.__dict__
