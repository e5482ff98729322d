#!/usr/bin/env python3
"""Debug: which parameters of the transformer DDP trainer (2 gloo ranks on one GPU) leave
sync, at which step."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import torch  # noqa: E402

from dist_utils import run_world  # noqa: E402


def worker(rank, world):
    import torch.distributed as dist
    from faster_distributed_training_amd.train.transformer_trainer import TransformerConfig, TransformerTrainer
    torch.cuda.set_device(0)
    cfg = TransformerConfig(batch_size=16, synthetic=True, eval=False, plot=False, distributed=True,
                            optimizer="mirror_madgrad", epoch=1, length_buckets=(128,), bucket_mb=4.0,
                            extra={"subset_stride": 50})
    tr = TransformerTrainer(cfg)
    if rank == 0:
        print("buckets", [(s, e, len(idx)) for s, e, idx in tr.reducer.buckets], flush=True)
    def cmp(tag, vals):
        alls = [torch.zeros_like(vals) for _ in range(world)]
        dist.all_gather(alls, vals)
        if rank == 0:
            bad = [(i, tr.flat.slots[i].name) for i in range(len(vals)) if alls[0][i] != alls[1][i]]
            print(f"{tag}: {len(bad)} of {len(vals)} differ: {bad[:6]}", flush=True)
    cmp("init params", torch.stack([s.param.detach().double().sum() for s in tr.flat.slots]).cpu())
    orig_step = tr.optimizer.step

    def spy(*a, **k):
        torch.cuda.synchronize()
        cmp("grads before optimizer", torch.stack([tr.flat.grad[s.offset:s.offset + s.numel].double().sum()
                                                  for s in tr.flat.slots]).cpu())
        cmp("shadow", torch.stack([tr.flat.shadow[s.offset:s.offset + s.numel].double().sum()
                                   for s in tr.flat.slots]).cpu())
        return orig_step(*a, **k)
    tr.optimizer.step = spy
    red = tr.reducer
    names = {id(sl.param): sl.name for sl in tr.flat.slots}
    log = []
    oh, ol = red._hook, red._launch

    class LogDict(dict):
        def __getitem__(self, k):
            b = dict.__getitem__(self, k)
            log.append(("ready", names[k], b, red.pending[b]))
            return b
    red.bucket_of = LogDict(red.bucket_of)

    def launch(b):
        log.append(("LAUNCH", b, red.pending[b]))
        return ol(b)
    red._launch = launch
    it = iter(tr.train_loader)
    for step in range(3):
        log.clear()
        tr.train_step(*next(it))
        torch.cuda.synchronize()
        if rank == 0 and step == 0:
            b4 = [e for e in log if (e[0] == "ready" and e[2] == 4) or e[0] == "LAUNCH"]
            print("events", len(log), [e for e in log if e[0] == "LAUNCH"], flush=True)
            print("bucket4 ready order", [(e[1][:40], e[3]) for e in b4 if e[0] == "ready"], flush=True)
        sums = torch.stack([s.param.detach().double().sum() for s in tr.flat.slots]).cpu()
        gs = torch.stack([tr.flat.grad[s.offset:s.offset + s.numel].double().sum() for s in tr.flat.slots]).cpu()
        alls = [torch.zeros_like(sums) for _ in range(world)]
        dist.all_gather(alls, sums)
        if rank == 0:
            bad = [(i, tr.flat.slots[i].name) for i in range(len(sums)) if alls[0][i] != alls[1][i]]
            print(f"step {step}: {len(bad)} params differ: {bad[:8]}", flush=True)


if __name__ == "__main__":
    run_world(worker, world=2, native=True, timeout=300)
