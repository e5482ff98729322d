"""DDP bucket reducer, flat-sharded FSDP, metric all-reduce and rank-0 checkpointing with
real multi-process gloo groups (world size 2 and 3) on the CPU."""
import os

import pytest
import torch
import torch.distributed as dist
import torch.nn as nn
import torch.nn.functional as F

from dist_utils import run_world


def _model(seed=0):
    torch.manual_seed(seed)
    return nn.Sequential(nn.Linear(10, 16), nn.ReLU(), nn.Linear(16, 12), nn.ReLU(), nn.Linear(12, 4))


def _batch(rank, n=8):
    g = torch.Generator().manual_seed(1000 + rank)
    return torch.randn(n, 10, generator=g), torch.randint(0, 4, (n,), generator=g)


def _ddp_worker(rank, world, bucket_mb):
    from faster_distributed_training_amd.parallel.ddp import BucketReducer
    from faster_distributed_training_amd.utils.flat import FlatParams
    m = _model(seed=rank)  # different init per rank: the reducer must broadcast rank 0's
    flat = FlatParams(m)
    red = BucketReducer(flat, m, bucket_mb=bucket_mb, first_bucket_mb=bucket_mb / 4)
    ref = _model(seed=0)
    for p, q in zip(m.parameters(), ref.parameters()):
        assert torch.equal(p, q)
    assert len(red.buckets) >= 2
    x, y = _batch(rank)
    F.cross_entropy(m(x), y).backward()
    red.finish()
    # reference: average of every rank's local gradient on the same (rank-0) weights
    grads = []
    for r in range(world):
        ref.zero_grad()
        xr, yr = _batch(r)
        F.cross_entropy(ref(xr), yr).backward()
        grads.append([p.grad.clone() for p in ref.parameters()])
    for i, p in enumerate(m.parameters()):
        avg = sum(g[i] for g in grads) / world
        assert torch.allclose(p.grad, avg, atol=1e-6), i


@pytest.mark.parametrize("world", [2, 3])
def test_bucket_reducer_averages_gradients(world):
    run_world(_ddp_worker, world=world, args=(0.0005,))


def _fsdp_worker(rank, world):
    from faster_distributed_training_amd.optim.flat_optim import SGD, GradClipper
    from faster_distributed_training_amd.parallel.fsdp import FlatShardedDP
    from faster_distributed_training_amd.utils.flat import FlatParams
    m = _model(seed=rank)
    flat = FlatParams(m)
    fs = FlatShardedDP(flat, m)
    opt = SGD(fs.view, lr=0.1, momentum=0.9)
    clip = GradClipper(fs.view, sharded=True)
    ref = _model(seed=0)
    ropt = torch.optim.SGD(ref.parameters(), lr=0.1, momentum=0.9)
    for step in range(3):
        x, y = _batch(rank + 10 * step)
        F.cross_entropy(m(x), y).backward()
        fs.finish_backward()
        clip(1.0)
        opt.step(grad_scale=clip.coef)
        fs.after_step()
        ropt.zero_grad()
        loss = sum(F.cross_entropy(ref(_batch(r + 10 * step)[0]), _batch(r + 10 * step)[1]) for r in range(world))
        (loss / world).backward()
        torch.nn.utils.clip_grad_norm_(ref.parameters(), 1.0)
        ropt.step()
        for p, q in zip(m.parameters(), ref.parameters()):
            assert torch.allclose(p, q, atol=1e-5), (step, (p - q).abs().max())


@pytest.mark.parametrize("world", [2, 3])
def test_flat_sharded_dp_matches_single_process(world):
    run_world(_fsdp_worker, world=world)


def _metrics_ckpt_worker(rank, world, path):
    from faster_distributed_training_amd.models import resnet as R
    from faster_distributed_training_amd.parallel.dist import all_reduce_metrics
    from faster_distributed_training_amd.train import checkpoint as ck
    a, b = torch.tensor([float(rank)]), torch.tensor([2.0 * rank + 1])
    all_reduce_metrics(a, b)
    assert a.item() == sum(range(world)) and b.item() == sum(2 * r + 1 for r in range(world))
    m = R.resnet18(10)
    ck.save_checkpoint(path, m, 12.5 + rank, 3, module_prefix=True)  # rank-0 writes, all barrier
    raw = torch.load(path, weights_only=True)
    assert raw["acc"] == 12.5  # written by rank 0 only


def test_metric_allreduce_and_rank0_checkpoint(tmp_path):
    run_world(_metrics_ckpt_worker, world=2, args=(str(tmp_path / "ck.pth"),))


def _trainer_worker(rank, world, tmp):
    from faster_distributed_training_amd.train.resnet_trainer import ResNetConfig, ResNetTrainer
    os.chdir(tmp)
    cfg = ResNetConfig(arch="resnet18", bs=4, synthetic=True, epoch=1, steps_per_epoch=2, eval=False, plot=False,
                       distributed=True, optimizer="sgd", extra={"subset_stride": 100})
    tr = ResNetTrainer(cfg)
    tr.fit()
    # every rank ends with identical parameters and BN running stats were synchronised
    flat = tr.flat.data.clone()
    other = flat.clone()
    dist.broadcast(other, 0)
    assert torch.allclose(flat, other)


def test_resnet_trainer_ddp_two_ranks(tmp_path):
    run_world(_trainer_worker, world=2, args=(str(tmp_path),))


def _eval_decision_worker(rank, world, tmp):
    """the "new best -> save" decision is collective (save_checkpoint barriers).
    Give each rank a different test set so local accuracies differ: every rank must still
    take rank 0's decision (no hang, same best_acc everywhere)."""
    from faster_distributed_training_amd.data.cifar import DeviceCIFARLoader, synthetic_cifar
    from faster_distributed_training_amd.train.resnet_trainer import ResNetConfig, ResNetTrainer
    os.chdir(tmp)
    cfg = ResNetConfig(arch="resnet18", bs=8, synthetic=True, epoch=1, steps_per_epoch=1, eval=True, plot=False,
                       distributed=True, optimizer="sgd", checkpoint_dir=os.path.join(tmp, "ck"),
                       extra={"subset_stride": 100})
    tr = ResNetTrainer(cfg)
    data, tg = synthetic_cifar(16, seed=50 + rank)
    tr.test_loader = DeviceCIFARLoader(data, tg, 8, tr.device, train=False, shuffle=False, drop_last=False)
    tr.best_acc = -1.0
    acc = tr.test(0)
    accs = [None] * world
    dist.all_gather_object(accs, (acc, tr.best_acc))
    assert all(a == accs[0] for a in accs), accs
    assert os.path.isfile(tr.ckpt_path)


def test_eval_save_decision_is_collective(tmp_path):
    run_world(_eval_decision_worker, world=2, args=(str(tmp_path),))


def _resume_rank_state_worker(rank, world, tmp):
    """per-rank RNG streams and (FSDP) per-rank optimizer shards survive
    save_last / auto-resume; rank 0's are not broadcast over the others."""
    from faster_distributed_training_amd.train import resilience
    from faster_distributed_training_amd.train.resnet_trainer import ResNetConfig, ResNetTrainer
    os.chdir(tmp)
    base = dict(arch="resnet18", bs=4, synthetic=True, epoch=1, steps_per_epoch=2, eval=False, plot=False,
                distributed=True, optimizer="madgrad", fsdp=True, checkpoint_dir=os.path.join(tmp, "ck"),
                extra={"subset_stride": 100})
    a = ResNetTrainer(ResNetConfig(save_last=True, **base)).fit()
    rng_after = torch.get_rng_state()
    opt_after = {k: v.clone() for k, v in a.optimizer.state_dict()["flat_state"].items() if torch.is_tensor(v)}
    assert os.path.isfile(resilience.rank_path(a.last_path, rank))
    torch.manual_seed(999)
    b = ResNetTrainer(ResNetConfig(auto_resume=True, **base))
    assert b.start_epoch == 1
    assert torch.equal(torch.get_rng_state(), rng_after)  # this rank's own stream
    opt_b = b.optimizer.state_dict()["flat_state"]
    assert all(torch.equal(opt_b[k], v) for k, v in opt_after.items())
    states = [None] * world
    dist.all_gather_object(states, torch.get_rng_state())
    assert not torch.equal(states[0], states[1])


def test_auto_resume_restores_each_ranks_state(tmp_path):
    run_world(_resume_rank_state_worker, world=2, args=(str(tmp_path),))
