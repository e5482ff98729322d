"""Deterministic mode (--deterministic, ops/_native.set_deterministic): two identical
ResNet engine steps give bitwise-identical logits, gradients and BN running statistics,
eager and replayed as HIP graphs (race detection: deterministic
reductions instead of shared fp32 atomics in the statistics kernels)."""
import pytest
import torch
import torch.nn.functional as F


def test_slot_rows_sizing():
    from faster_distributed_training_amd.ops import _native
    from faster_distributed_training_amd.ops import conv_igemm as ci
    assert ci.slot_rows() == ci.STAT_SLOTS
    _native.set_deterministic(True)
    try:
        assert ci.slot_rows(128) == ci.STAT_SLOTS  # at least the shared-slot count (det mode)
        assert ci.slot_rows(64 * 100) == 128       # one row per 64-row block, power of two
        assert ci.slot_rows(1024 * 32 * 32) == 16384
        with pytest.raises(AssertionError):
            ci.slot_rows()
    finally:
        _native.set_deterministic(False)
    assert not _native.deterministic()


@pytest.fixture
def det_mode():
    from faster_distributed_training_amd.ops import _native
    _native.set_deterministic(True)
    yield
    _native.set_deterministic(False)


def _run_steps(cuda, arch, batch, graphs, n):
    from faster_distributed_training_amd.models import resnet as R
    from faster_distributed_training_amd.utils.flat import FlatParams
    torch.manual_seed(0)
    m = getattr(R, arch)(10).to(cuda)
    m.fast_path = True
    m.graph_engine = graphs
    flat = FlatParams(m, device=cuda)
    g = torch.Generator().manual_seed(5)
    x = torch.randn(batch, 3, 32, 32, generator=g).to(cuda)
    y = torch.randint(0, 10, (batch,), generator=g).to(cuda)
    buf0 = [b.detach().clone() for b in m.buffers()]
    outs = []
    for _ in range(n):
        # identical starting state every step: same weights (no optimizer step), same
        # running statistics (restored in place, graph-safe)
        for b, b0 in zip(m.buffers(), buf0):
            b.copy_(b0)
        flat.grad.zero_()
        out = m(x)
        F.cross_entropy(out.float(), y).backward()
        torch.cuda.synchronize()
        outs.append((out.detach().clone(), flat.grad.clone(), [b.detach().clone() for b in m.buffers()]))
    return outs


def _bitwise(a, b):
    ints = {1: torch.uint8, 2: torch.int16, 4: torch.int32, 8: torch.int64}
    return a.dtype == b.dtype and a.shape == b.shape and \
        torch.equal(a.view(ints[a.element_size()]), b.view(ints[b.element_size()]))


@pytest.mark.gpu
@pytest.mark.parametrize("arch,batch", [("resnet50", 64), ("resnet18", 48)])
def test_deterministic_steps_bitwise(cuda, det_mode, arch, batch):
    eager = _run_steps(cuda, arch, batch, graphs=False, n=2)
    graphed = _run_steps(cuda, arch, batch, graphs=True, n=4)  # warm-up, capture, 2 replays
    ref = eager[0]
    for run in eager[1:] + graphed:
        assert _bitwise(run[0], ref[0]), "logits differ"
        assert _bitwise(run[1], ref[1]), "gradients differ"
        for b, rb in zip(run[2], ref[2]):
            assert _bitwise(b, rb), "running statistics differ"
