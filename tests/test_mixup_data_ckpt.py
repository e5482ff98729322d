"""Mixup family, CIFAR data path and checkpoint schema (CPU)."""
import os

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from faster_distributed_training_amd.data import cifar as C
from faster_distributed_training_amd.models import resnet as R
from faster_distributed_training_amd.ops import mixup as M
from faster_distributed_training_amd.train import checkpoint as ck


def test_mixup_data_interpolates():
    torch.manual_seed(0)
    x = torch.randn(8, 3, 4, 4)
    y = torch.arange(8)
    g = torch.Generator().manual_seed(1)
    mixed, ya, yb, lam = M.mixup_data(x, y, alpha=0.99, generator=g)
    assert 0.0 <= lam <= 1.0
    perm = yb  # labels are arange, so y[perm] == perm
    assert torch.allclose(mixed, lam * x + (1 - lam) * x[perm], atol=1e-6)
    assert torch.equal(ya, y)


def test_mixup_alpha_nonpositive_is_fixed_lambda():
    assert M.sample_lambda(0.0) == 0.0 and M.sample_lambda(-0.5) == -0.5


def test_mixup_intra_only_keeps_same_label_pairs():
    x = torch.randn(6, 2)
    y = torch.tensor([0, 0, 0, 0, 0, 0])
    mixed, ya, yb, lam = M.mixup_data(x, y, alpha=0.5, intra_only=True)
    assert torch.allclose(mixed, x)  # every pair has the same label -> no mixing


def test_mixup_criteria():
    torch.manual_seed(0)
    logits = torch.randn(5, 10, requires_grad=True)
    ya, yb = torch.randint(0, 10, (5,)), torch.randint(0, 10, (5,))
    lam = 0.3
    l = M.mixup_criterion(None, logits, ya, yb, lam)
    ref = lam * F.cross_entropy(logits, ya) + (1 - lam) * F.cross_entropy(logits, yb)
    assert torch.allclose(l, ref, atol=1e-6)
    lv = torch.rand(5, 1, 1, 1)
    lm = M.mixup_criterion_meta(None, logits, ya, yb, lv)
    ref_m = (lv.view(5) * F.cross_entropy(logits, ya, reduction="none") +
             (1 - lv.view(5)) * F.cross_entropy(logits, yb, reduction="none")).mean()
    assert torch.allclose(lm, ref_m, atol=1e-6)
    # faithful: the reference's (B,1,1,B) broadcast equals the mean-lambda form
    lf = M.mixup_criterion_meta(None, logits, ya, yb, lv, faithful=True)
    ce_a = F.cross_entropy(logits, ya, reduction="none")
    ce_b = F.cross_entropy(logits, yb, reduction="none")
    broadcast = (lv * ce_a + (1 - lv) * ce_b).mean()  # the reference's shape (B,1,1,B)
    assert torch.allclose(lf, broadcast, atol=1e-6)


def test_meta_mixup_faithful_and_learnable():
    m = M.MetaMixup(4)
    x, y = torch.randn(4, 3, 2, 2), torch.arange(4)
    t0 = m.lam.detach().clone()
    mixed, ya, yb, lam = m(x, y)
    assert not torch.equal(t0, m.lam)  # faithful: resampled each step (reference Q3)
    assert lam.shape == (4, 1, 1, 1) and torch.all((lam >= 0.5) & (lam <= 0.7311))
    ml = M.MetaMixup(4, learnable=True)
    t1 = ml.lam.detach().clone()
    _, _, _, lam = ml(x, y)
    assert torch.equal(t1, ml.lam.detach()) and ml.lam.requires_grad


def test_augment_cpu_shapes_and_eval_normalise_only():
    imgs = torch.randint(0, 256, (4, 32, 32, 3), dtype=torch.uint8)
    x = C.augment_cpu(imgs, torch.Generator().manual_seed(0), train=False)
    ref = (imgs.permute(0, 3, 1, 2).float() / 255 - torch.tensor(C.CIFAR_MEAN).view(1, 3, 1, 1)) / \
        torch.tensor(C.CIFAR_STD).view(1, 3, 1, 1)
    assert torch.allclose(x, ref, atol=1e-6)
    xt = C.augment_cpu(imgs, torch.Generator().manual_seed(0), train=True)
    assert xt.shape == (4, 3, 32, 32)


def test_loader_sharding_set_epoch_drop_last():
    data, targets = C.synthetic_cifar(100, seed=0)
    seen = []
    for r in range(2):
        ld = C.DeviceCIFARLoader(data, targets, 8, "cpu", rank=r, world_size=2, seed=3)
        assert len(ld) == 50 // 8
        idx = ld._indices()
        seen.append(set(idx.tolist()))
        ld.set_epoch(1)
        assert not torch.equal(idx, ld._indices())  # Q10: new shuffle per epoch
    assert not (seen[0] & seen[1])  # disjoint shards
    ld = C.DeviceCIFARLoader(data, targets, 8, "cpu", train=False, shuffle=False, drop_last=False)
    n = sum(b[0].shape[0] for b in ld)
    assert n == 100


def test_cifar_pickle_loader_rejects_code(tmp_path):
    import pickle
    bad = tmp_path / "data_batch_1"
    with open(bad, "wb") as f:
        pickle.dump({"x": os.system}, f)
    with pytest.raises(Exception):
        C._load_batch(str(bad))


def test_checkpoint_reference_schema_roundtrip(tmp_path):
    m = R.resnet18(10)
    p = tmp_path / "checkpoint" / "resnet_ckpt.pth"
    ck.save_checkpoint(str(p), m, 91.5, 7, module_prefix=True)
    raw = torch.load(str(p), weights_only=True)
    assert set(raw) == {"net", "acc", "epoch"} and raw["acc"] == 91.5 and raw["epoch"] == 7
    assert all(k.startswith("module.") for k in raw["net"])
    m2 = R.resnet18(10)
    ck.load_model_state(m2, raw["net"])
    for a, b in zip(m.state_dict().values(), m2.state_dict().values()):
        assert torch.equal(a, b)
    best, start = ck.load_best_performance(str(p), 10, resume=True)
    assert best == 91.5 and start == 7
    assert ck.load_best_performance(str(p), 10, resume=False) == (0.1, 0)


def test_checkpoint_loads_into_flat_model(tmp_path):
    from faster_distributed_training_amd.utils.flat import FlatParams
    m = R.resnet18(10)
    flat = FlatParams(m)
    src = R.resnet18(10)
    path = tmp_path / "c.pth"
    ck.save_checkpoint(str(path), src, 50.0, 1)
    ck.load_model_state(m, torch.load(str(path), weights_only=True)["net"])
    # parameters stay views into the flat buffer
    p0 = next(m.parameters())
    assert p0.data_ptr() == flat.data[flat.slot_of(p0).offset:].data_ptr()
    assert torch.equal(p0, next(src.parameters()))


def test_faithful_augment_order_and_padding():
    """Q13: --faithful draws the transform permutation once from the run seed; only the
    position of Normalize relative to the padded crop is observable (padding value)."""
    from faster_distributed_training_amd.data import cifar as C
    assert C.augment_order(1, faithful=False) == ("crop", "flip", "normalize")
    orders = {C.augment_order(s, faithful=True) for s in range(40)}
    assert len(orders) == 6 and C.augment_order(5, True) == C.augment_order(5, True)
    imgs = torch.full((16, 32, 32, 3), 128, dtype=torch.uint8)
    for order in (("crop", "flip", "normalize"), ("normalize", "flip", "crop")):
        x = C.augment_cpu(imgs, torch.Generator().manual_seed(0), train=True, order=order)
        pad = 0.0 if C.pad_normalized(order) else -C.CIFAR_MEAN[0] / C.CIFAR_STD[0]
        inside = (128 / 255 - C.CIFAR_MEAN[0]) / C.CIFAR_STD[0]
        v = x[:, 0]
        assert bool((((v - pad).abs() < 1e-5) | ((v - inside).abs() < 1e-5)).all())


def test_skipped_steps_do_not_advance_madgrad_counter():
    """a step skipped on non-finite gradients must not advance MADGRAD's k
    (torch GradScaler never calls optimizer.step() on it)."""
    from faster_distributed_training_amd.optim.flat_optim import MADGRAD
    from faster_distributed_training_amd.utils.flat import FlatParams

    def run(skip):
        torch.manual_seed(0)
        m = torch.nn.Linear(4, 3)
        flat = FlatParams(m)
        opt = MADGRAD(flat, lr=0.1)
        for i in range(3):
            torch.manual_seed(10 + i)
            m(torch.randn(5, 4)).square().sum().backward()
            opt.step(found_inf=torch.zeros(1, dtype=torch.int32))
            if skip and i == 0:
                flat.grad.fill_(float("inf"))
                opt.step(found_inf=torch.ones(1, dtype=torch.int32))
        return flat.data.clone(), opt
    a, _ = run(False)
    b, ob = run(True)
    assert ob.k == 4 and ob.applied_k == 3
    assert torch.equal(a, b)
