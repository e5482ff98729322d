"""Debug: sharded vs unsharded NGD trainer runs (world 1, RCCL, graphs, deterministic) --
per-key max parameter differences after K steps, with/without the fused head."""
import os
import sys

os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
os.environ.setdefault("MASTER_PORT", "29533")
os.environ.setdefault("RANK", "0")
os.environ.setdefault("LOCAL_RANK", "0")
os.environ.setdefault("WORLD_SIZE", "1")
os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import torch.distributed as dist

torch.cuda.set_device(0)
dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
from faster_distributed_training_amd.ops import resnet_fused as rf
from faster_distributed_training_amd.train.resnet_trainer import ResNetConfig, ResNetTrainer

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 5


def run(sharded, head, graphs=True, det=True):
    rf.FUSED_HEAD = head
    base = dict(arch="resnet18", bs=32, synthetic=True, eval=False, plot=False, ngd=True, optimizer="ngd",
                deterministic=det, graphs=graphs, extra={"subset_stride": 50})
    tr = ResNetTrainer(ResNetConfig(force_sharded=sharded, bucket_mb=2.0, first_bucket_mb=0.5, **base))
    it = iter(tr.train_loader)
    out = []
    grads = []
    orig = tr.optimizer.step

    def step(*a, **k):
        torch.cuda.synchronize()
        d = {n: p.grad.detach().float().clone() for n, p in tr.model.named_parameters()}
        sp = tr.space
        for sl in sp.slots:
            d["SPACE." + sl.name] = sp.grad[sl.offset:sl.offset + sl.numel].float().clone()
        d["CLIP.coef"] = tr.clipper.coef.detach().float().clone().reshape(-1)
        d["CLIP.out"] = tr.clipper.out.detach().float().clone().reshape(-1)
        grads.append(d)
        return orig(*a, **k)
    tr.optimizer.step = step
    for i in range(steps):
        x, y = next(it)
        tr.train_step(x, y)
        torch.cuda.synchronize()
        out.append({k: v.detach().float().clone() for k, v in tr.model.state_dict().items() if v.dtype.is_floating_point})
    print("head_on", sharded, head, graphs, getattr(tr.model._plan, "head_on", None), flush=True)
    return out, grads


def cmp(name, a, b):
    for i, (sa, sb) in enumerate(zip(a, b)):
        d = {k: (sa[k] - sb[k]).abs().max().item() for k in sa}
        bad = [(k, v) for k, v in d.items() if v > 0]
        worst = sorted(bad, key=lambda kv: -kv[1])[:3]
        print(f"{name} step {i}: {len(bad)}/{len(d)} keys differ; worst {worst}", flush=True)


u1, gu1 = run(False, True)
s1, gs1 = run(True, True)
u0, gu0 = run(False, False)
s0, gs0 = run(True, False)
cmp("head: unsharded vs sharded", u1, s1)
cmp("GRAD head: unsharded vs sharded", gu1, gs1)
cmp("GRAD nohead: unsharded vs sharded", gu0, gs0)
cmp("GRAD sharded: head vs nohead", gs1, gs0)
cmp("GRAD unsharded: head vs nohead", gu1, gu0)
dist.destroy_process_group()
