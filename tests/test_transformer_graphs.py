"""Transformer forward+backward as a replayed HIP graph (train/transformer_trainer.py)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _trainer(graphs, monkeypatch, **kw):
    import faster_distributed_training_amd.train.transformer_trainer as T
    monkeypatch.setattr(T, "TR_GRAPHS", graphs)
    cfg = T.TransformerConfig(batch_size=32, synthetic=True, eval=False, plot=False, ngd=False, optimizer="sgd",
                              epoch=1, steps_per_epoch=8, length_buckets=(128,), extra={"subset_stride": 50},
                              n_layers=2, **kw)
    return T.TransformerTrainer(cfg)


def test_graph_replay_matches_eager(cuda, monkeypatch):
    """Dropout off and lambda = 0 (mixup with the permuted labels: the batch-mean loss and
    its gradient do not depend on the permutation), so eager and graphed runs compute the
    same trajectory: 2 side-stream warm-up steps, capture + replay, then replays."""
    import torch.nn as nn

    def run(graphs):
        torch.manual_seed(0)
        tr = _trainer(graphs, monkeypatch)
        for mod in tr.model.modules():
            if isinstance(mod, nn.Dropout):
                mod.p = 0.0
        tr.model.alpha = 0.0
        it = iter(tr.train_loader)
        losses = [float(tr.train_step(*next(it))) for _ in range(6)]
        torch.cuda.synchronize()
        return losses, tr.space.data.clone(), tr

    le, pe, _ = run(False)
    lg, pg, tg = run(True)
    assert any(isinstance(v, dict) for v in tg._graphs.values()), "graph path not taken"
    assert max(abs(a - b) / max(abs(a), 1e-6) for a, b in zip(le, lg)) < 1e-3, (le, lg)
    assert ((pe - pg).norm() / pe.norm()).item() < 1e-4


def test_attention_device_seed_redraws_dropout(cuda):
    """The per-replay device seed changes the attention dropout mask; the same seed
    reproduces it (forward and the regenerated mask in backward agree: grads finite)."""
    from faster_distributed_training_amd.ops import attention_native as AN
    torch.manual_seed(0)
    q, k, v = [torch.randn(2, 64, 4, 64, device=cuda, dtype=torch.bfloat16, requires_grad=True) for _ in range(3)]
    seed = torch.zeros(1, dtype=torch.int64, device=cuda)
    AN.DEVICE_SEED = seed
    try:
        torch.manual_seed(1)
        a = AN.attention_native(q, k, v, dropout_p=0.3)
        torch.manual_seed(1)
        b = AN.attention_native(q, k, v, dropout_p=0.3)
        seed.fill_(12345)
        torch.manual_seed(1)
        c = AN.attention_native(q, k, v, dropout_p=0.3)
        c.float().sum().backward()
    finally:
        AN.DEVICE_SEED = None
    assert torch.equal(a, b)
    assert not torch.equal(a, c)
    assert all(torch.isfinite(t.grad).all() for t in (q, k, v))


def test_shadow_weights_match_casts(cuda, monkeypatch):
    """bf16 shadow weights (rewritten by the optimizer kernel) give the same trajectory as
    casting the fp32 master weights each forward (graphs off, dropout off)."""
    import torch.nn as nn
    import faster_distributed_training_amd.train.transformer_trainer as T

    def run(shadow):
        monkeypatch.setattr(T, "SHADOW", shadow)
        torch.manual_seed(0)
        tr = _trainer(False, monkeypatch)
        assert (tr.flat.shadow is not None) == shadow
        for mod in tr.model.modules():
            if isinstance(mod, nn.Dropout):
                mod.p = 0.0
        tr.model.alpha = 0.0
        it = iter(tr.train_loader)
        losses = [float(tr.train_step(*next(it))) for _ in range(4)]
        torch.cuda.synchronize()
        return losses, tr.flat.data.clone()

    lc, pc = run(False)
    ls, ps = run(True)
    assert max(abs(a - b) / max(abs(a), 1e-6) for a, b in zip(lc, ls)) < 1e-3, (lc, ls)
    assert ((pc - ps).norm() / pc.norm()).item() < 1e-4
