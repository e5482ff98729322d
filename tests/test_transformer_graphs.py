"""Transformer forward+backward as a replayed HIP graph (train/transformer_trainer.py)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _trainer(graphs, monkeypatch, **kw):
    import faster_distributed_training_amd.train.transformer_trainer as T
    monkeypatch.setattr(T, "TR_GRAPHS", graphs)
    extra = kw.pop("extra", {"subset_stride": 50})
    cfg = T.TransformerConfig(batch_size=32, synthetic=True, eval=False, plot=False, ngd=False, optimizer="sgd",
                              epoch=1, steps_per_epoch=8, length_buckets=(128,), extra=extra,
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


def test_torch_op_step_graph_replay_matches_eager(cuda, monkeypatch):
    """Review r2 5a: the --no-native (plain torch ops) transformer step captured as a HIP
    graph used to fault on replay (aperture violation in rocprim partition_kernel: ATen's
    dense embedding backward sizes its unique-by-key buffers from a value read at capture
    time).  With the static-shape index_add embedding backward the captured torch-op step
    replays to the eager trajectory; the capture guard is active during capture."""
    import torch.nn as nn
    monkeypatch.setenv("FDT_NATIVE", "0")

    def run(graphs):
        torch.manual_seed(0)
        tr = _trainer(graphs, monkeypatch, extra={"subset_stride": 50, "graphs_torch_ops": True})
        for mod in tr.model.modules():
            if isinstance(mod, nn.Dropout):
                mod.p = 0.0
        tr.model.alpha = 0.0
        assert tr._graphs_on() == graphs
        it = iter(tr.train_loader)
        losses = [float(tr.train_step(*next(it))) for _ in range(6)]
        torch.cuda.synchronize()
        return losses, tr.space.data.clone(), tr

    le, pe, _ = run(False)
    lg, pg, tg = run(True)
    assert any(isinstance(v, dict) for v in tg._graphs.values()), "graph path not taken"
    assert max(abs(a - b) / max(abs(a), 1e-6) for a, b in zip(le, lg)) < 1e-3, (le, lg)
    assert ((pe - pg).norm() / pe.norm()).item() < 1e-4


def test_capture_guard_refuses_data_dependent_ops(cuda):
    """Inside a capture, ops with data-dependent output sizes raise instead of recording a
    capture-time size (forward and autograd backward)."""
    from faster_distributed_training_amd.parallel.graphs import CaptureUnsafeOp, capture_guard
    x = torch.randn(64, device=cuda)
    w = torch.randn(10, 8, device=cuda, requires_grad=True)
    idx = torch.randint(0, 10, (32,), device=cuda)
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        with pytest.raises(CaptureUnsafeOp):
            with torch.cuda.graph(g, stream=s), capture_guard():
                torch.nonzero(x > 0)
    out = torch.nn.functional.embedding(idx, w).sum()
    with pytest.raises(CaptureUnsafeOp):
        with capture_guard():
            out.backward()


def test_graph_step_accumulates_meter_in_loss_kernel(cuda, monkeypatch):
    """The replayed step's loss kernel adds the loss / lambda-weighted accuracy into the
    DeviceMeter (no per-step accuracy kernels); the meter's buffer keeps its address across
    resets.  Its loss sum equals the sum of the returned step losses, over warm-up, capture
    and replays alike, and every sample is counted once."""
    tr = _trainer(True, monkeypatch)
    it = iter(tr.train_loader)
    acc_ptr = tr.meter.acc.data_ptr()
    losses = []
    for _ in range(6):
        losses.append(float(tr.train_step(*next(it))))
    torch.cuda.synchronize()
    assert any(isinstance(v, dict) and v.get("meter") for v in tr._graphs.values()), "fused meter not captured"
    loss_sum, correct, total = tr.meter.acc.tolist()
    assert abs(loss_sum - sum(losses)) <= 1e-4 * max(1.0, abs(sum(losses))), (loss_sum, losses)
    assert total == 6 * 32 and 0.0 <= correct <= total
    assert tr.meter.steps == 6
    tr.meter.reset()
    assert tr.meter.acc.data_ptr() == acc_ptr and float(tr.meter.acc.abs().sum()) == 0.0
