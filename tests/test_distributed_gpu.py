"""The fused ResNet engine under the DDP bucket reducer, two ranks (gloo, both on cuda:0).

Every gradient is snapshotted at the moment it becomes ready (a grad-ready / post-
accumulate hook registered before the reducer's), i.e. before its bucket is reduced in
place.  Checks: the engine's hooks launch every bucket during backward; the reduced
gradient equals the average of the per-rank snapshots; all ranks hold the same result.
(The engine's BN statistics use fp32 atomics, so two runs of the same batch are not
bitwise equal -- comparing against a separate single-process run would test noise.)"""
import pytest
import torch
import torch.nn.functional as F

from dist_utils import run_world

pytestmark = pytest.mark.gpu


def _batch(rank, n=16):
    g = torch.Generator().manual_seed(500 + rank)
    return torch.randn(n, 3, 32, 32, generator=g), torch.randint(0, 10, (n,), generator=g)


def _worker(rank, world):
    import torch.distributed as dist
    from faster_distributed_training_amd.models import resnet as R
    from faster_distributed_training_amd.ops.resnet_fused import register_grad_ready_hook
    from faster_distributed_training_amd.parallel.ddp import BucketReducer
    from faster_distributed_training_amd.utils.flat import FlatParams
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    torch.manual_seed(rank)  # different init per rank: the reducer broadcasts rank 0's
    m = R.resnet50(10).to(dev)
    m.fast_path = True
    flat = FlatParams(m, device=dev)
    snap = {}

    def take(p):
        snap[id(p)] = p.grad.detach().clone()

    for p in m.parameters():
        register_grad_ready_hook(p, take)
        p.register_post_accumulate_grad_hook(take)
    red = BucketReducer(flat, m, bucket_mb=4.0, first_bucket_mb=0.5)
    assert len(red.buckets) >= 4
    x, y = _batch(rank)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        out = m(x.to(dev))
    F.cross_entropy(out.float(), y.to(dev)).backward()
    assert all(w is not None for w in red.works), "a bucket was never launched by the hooks"
    red.finish()
    assert len(snap) == len(list(m.parameters()))
    local = torch.zeros_like(flat.grad)
    for s in flat.slots:
        local[s.offset:s.offset + s.numel] = snap[id(s.param)].reshape(-1)
    mean = local.clone()
    dist.all_reduce(mean)
    mean /= world
    err = ((flat.grad - mean).norm() / mean.norm()).item()
    assert err < 1e-6, err
    assert ((local - mean).norm() / mean.norm()).item() > 1e-3  # the ranks really differed
    chk = torch.tensor([flat.grad.double().sum().item(), flat.grad.abs().double().sum().item()])
    alls = [torch.zeros_like(chk) for _ in range(world)]
    dist.all_gather(alls, chk)
    assert all(torch.equal(alls[0], t) for t in alls)


def test_ddp_engine_two_ranks_one_gpu(cuda):
    run_world(_worker, world=2, native=True, timeout=400)


def _graph_worker(rank, world):
    import torch.distributed as dist
    from faster_distributed_training_amd.models import resnet as R
    from faster_distributed_training_amd.parallel.ddp import BucketReducer
    from faster_distributed_training_amd.utils.flat import FlatParams
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    torch.manual_seed(rank)
    m = R.resnet50(10).to(dev)
    m.fast_path = True
    m.graph_engine = True
    flat = FlatParams(m, device=dev)
    red = BucketReducer(flat, m, bucket_mb=4.0, first_bucket_mb=0.5)
    x, y = _batch(rank)
    for it in range(4):
        flat.grad.zero_()
        with torch.autocast("cuda", dtype=torch.bfloat16):
            out = m(x.to(dev))
        F.cross_entropy(out.float(), y.to(dev)).backward()
        assert all(w is not None for w in red.works), (it, "bucket not launched")
        red.finish()
        assert torch.isfinite(flat.grad).all()
        chk = torch.tensor([flat.grad.double().sum().item()])
        alls = [torch.zeros_like(chk) for _ in range(world)]
        dist.all_gather(alls, chk)
        assert all(torch.equal(alls[0], t) for t in alls), it
    st = list(m._plan._graphs.values())[0]
    assert st.stage == "ready" and len(st.segments) > 2  # backward cut at bucket boundaries


def test_ddp_engine_hip_graphs_two_ranks(cuda):
    run_world(_graph_worker, world=2, native=True, timeout=400)
