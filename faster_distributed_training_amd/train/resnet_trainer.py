"""ResNet / CIFAR-10 training driver (reference ``resnet50_test.py:460-740``; T1, T2, T5).

Per step (all on device, no host synchronisation):
  batch (device-resident CIFAR + GPU augment) -> mixup (A1) or meta-mixup (A2) ->
  forward (HIP engine, bf16) -> fused mixup cross-entropy -> backward (DDP buckets
  all-reduced on RCCL while backward runs) -> clip-norm coefficient on device ->
  one fused optimizer launch (MADGRAD / SGD / NGD / Adam) -> device-side metrics.
Per epoch: metric all-reduce (one collective), scheduler step, eval, rank-0
best checkpoint in the reference schema, JSONL log, plots at the end.
"""
from __future__ import annotations

import math
import os
import time
from dataclasses import dataclass, field

import numpy as np
import torch
import torch.nn as nn

from ..data.cifar import CLASSES, CIFAR10, DeviceCIFARLoader, augment_order, synthetic_cifar
from ..models import resnet as resnet_models
from ..ops.mixup import unit_grad, MetaMixup, mixup_criterion, mixup_criterion_meta, mixup_data
from ..ops.resnet_fused import STAGES
from ..optim.flat_optim import MADGRAD, SGD, Adam, DeviceGradScaler, GradClipper, MirrorMADGRAD
from ..optim.ngd import NGD
from ..parallel import dist as pdist
from ..utils.env import default_device, print0, seed_everything
from ..utils.flat import FlatParams
from . import checkpoint as ckpt
from . import resilience
from .metrics import DeviceMeter, JsonlLogger, PhaseProfiler, draw_graph, peak_memory_gb


@dataclass
class ResNetConfig:
    arch: str = "resnet50"
    num_classes: int = 10
    bs: int = 128                      # per process (reference --bs)
    lr: float = 0.02
    epoch: int = 50
    alpha: float = 0.99                # Beta(alpha, alpha) for mixup
    meta_learning: bool = False
    learnable_meta: bool = False       # Q3 fix: optimise the meta-mixup lambda
    distributed: bool = False
    ngd: bool = False
    optimizer: str = "auto"            # auto: ngd->NGD, else MADGRAD (reference defaults)
    weight_decay: float | None = None  # auto: NGD 1e-4, MADGRAD 5e-6, SGD 5e-4
    momentum: float = 0.9
    clip: float = 10.0
    precision: str = "bf16"            # bf16 | fp16 (GradScaler) | fp32
    synthetic: bool = False
    data_root: str = "./data"
    seed: int = 123456
    faithful: bool = False
    lr_scaling: str = "world"          # world | faithful4 | none   (Q11)
    bucket_mb: float = 25.0           # DDP / ZeRO-2 buckets (parallel/ddp.py: bucket sizing)
    first_bucket_mb: float = 1.0
    comm_dtype: str = "fp32"
    fsdp: bool = False
    fsdp_offload: bool = False         # FSDP shards + optimizer state in pinned host memory (CPUOffload)
    fsdp_offload_optimizer: str = "device"  # "device": optimizer on the GPU over the staged shard; "host": on the CPU
    fsdp_param_dtype: str = "fp32"     # fp32 | bf16: all-gather wire / compute copy of the parameters
    fsdp_schedule: str = "full_shard"  # full_shard (reshard after forward) | shard_grad_op (graph path only)
    shard_ngd: bool = True             # distributed NGD: each rank owns + preconditions 1/world of the params
    scheduler: str = "auto"
    resume: bool = False
    checkpoint_dir: str = "./checkpoint"
    steps_per_epoch: int = 0           # 0 = full epoch
    eval: bool = True
    log_path: str | None = None
    plot: bool = True
    workers: int = 2                   # accepted for CLI parity (no worker processes needed)
    fast_path: bool | None = None      # None = HIP engine when on GPU
    graphs: bool = True                # run the engine body as captured HIP graphs (train steps)
    auto_resume: bool = False          # restore *_last.pth (full state) if present; implies save_last
    save_last: bool = False            # write the rolling full-state *_last.pth every epoch
    nonfinite_guard: bool = True       # skip (on device) optimizer steps whose gradients are not finite
    profile_steps: int = 0             # per-phase device timing (+ roctx ranges) of the first K steps
    deterministic: bool = False        # bitwise-repeatable engine steps (ops/_native.set_deterministic)
    force_sharded: bool = False        # sharded-NGD path even at world size 1 (bench / tests)
    force_ddp: bool = False            # DDP bucket reducer even at world size 1 (bench: the 8-GPU
                                       # path's graph cuts + all-reduce actions on one GPU)
    extra: dict = field(default_factory=dict)


def build_model(cfg: ResNetConfig, device):
    model = getattr(resnet_models, cfg.arch)(cfg.num_classes)
    model.fast_path = cfg.fast_path
    model.graph_engine = cfg.graphs
    return model.to(device)


class ResNetTrainer:
    def __init__(self, cfg: ResNetConfig):
        self.cfg = cfg
        self.rank, self.world = 0, 1
        if (cfg.distributed or cfg.fsdp or cfg.force_sharded or cfg.force_ddp
                or int(os.environ.get("WORLD_SIZE", "1")) > 1):
            # (--fsdp always runs the sharded path, over a world-1 group on one GPU)
            if not torch.distributed.is_initialized():
                pdist.setup_norank()
            self.rank, self.world = pdist.rank(), pdist.world()
            cfg.distributed = self.world > 1
        self.device = default_device()
        if cfg.deterministic:
            from ..ops import _native
            _native.set_deterministic(True)
        seed_everything(cfg.seed)  # identical init on every rank
        self.model = build_model(cfg, self.device)
        self.best_acc, self.start_epoch = ckpt.load_best_performance(self.ckpt_path, cfg.num_classes, cfg.resume)
        if cfg.resume:
            ck = ckpt.load_checkpoint(self.ckpt_path)
            ckpt.load_model_state(self.model, ck["net"])
        self.meta = None
        if cfg.meta_learning:
            self.meta = MetaMixup(cfg.bs, device=self.device, learnable=cfg.learnable_meta)
        learnable = bool(self.meta and cfg.learnable_meta)
        params_owner = self.model if not learnable else nn.ModuleList([self.model, self.meta])
        ngd_opt = cfg.optimizer == "ngd" or (cfg.optimizer == "auto" and cfg.ngd)
        self.reducer = self.fsdp = self.zero = None
        if cfg.fsdp:
            # ZeRO-3: parameters sharded at rest, gathered per stage (parallel/fsdp.py); NGD
            # needs whole parameters per rank ("param" shard mode, survey Q17)
            if learnable:
                raise ValueError("--fsdp does not shard the learnable meta-mixup parameters")
            from ..parallel.fsdp import FullyShardedDP
            engine = self.model.use_fast_path(torch.empty(1, device=self.device))
            # HIP graphs under FSDP: static mode (fixed-address unit buffers, collectives between
            # graph segments) -- FULL_SHARD on a two-slot ring (default) or SHARD_GRAD_OP with
            # every unit's buffers persistent; eager FSDP is the full ZeRO-3 schedule
            static = bool(engine and cfg.graphs and not cfg.fsdp_offload and cfg.extra.get("fsdp_static", True))
            if cfg.fsdp_schedule not in ("full_shard", "shard_grad_op"):
                raise ValueError(f"fsdp_schedule {cfg.fsdp_schedule!r}")
            self.model.graph_engine = static
            self.fsdp = FullyShardedDP(self.model, self.device, mode="param" if ngd_opt else "flat",
                                       offload=cfg.fsdp_offload, static=static,
                                       offload_optimizer="host" if cfg.faithful else cfg.fsdp_offload_optimizer,
                                       reshard_after_forward=cfg.fsdp_schedule == "full_shard",
                                       param_dtype={"fp32": None, "bf16": torch.bfloat16}[cfg.fsdp_param_dtype],
                                       engine_units=("conv1",) + STAGES if engine else ())
            if engine:
                self.model._fsdp = self.fsdp
            self.flat = self.fsdp.space
        elif (cfg.distributed or cfg.force_sharded) and ngd_opt and cfg.shard_ngd:
            # ZeRO-2 for NGD: each rank preconditions + updates only the parameters it owns
            # (parallel/zero.py) instead of every rank repeating the whole NGD step
            from ..parallel.zero import ShardedOptimizerDP
            self.flat = FlatParams(params_owner, device=self.device, partition=self.world, balance="ngd")
            cdt = {"fp32": None, "bf16": torch.bfloat16}[cfg.comm_dtype]
            self.zero = ShardedOptimizerDP(self.flat, self.model, bucket_mb=cfg.bucket_mb,
                                           first_bucket_mb=cfg.first_bucket_mb, comm_dtype=cdt)
        else:
            self.flat = FlatParams(params_owner, device=self.device)
            # SGD / MADGRAD steps write the engine's packed conv weights (ops/resnet_fused.py)
            self.flat.pack_owner = self.model
            if cfg.distributed or cfg.force_ddp:
                from ..parallel.ddp import BucketReducer
                cdt = {"fp32": None, "bf16": torch.bfloat16}[cfg.comm_dtype]
                self.reducer = BucketReducer(self.flat, self.model, bucket_mb=cfg.bucket_mb,
                                             first_bucket_mb=cfg.first_bucket_mb, comm_dtype=cdt)
        self.sharder = self.fsdp if self.fsdp is not None else self.zero
        seed_everything(cfg.seed, self.rank)  # per-rank data/mixup randomness
        self.space = self.sharder.view if self.sharder is not None else self.flat
        self.optimizer, self.scheduler = self._build_optimizer()
        self.clipper = GradClipper(self.space, sharded=self.sharder is not None)
        self.scaler = DeviceGradScaler(self.device, enabled=(cfg.precision == "fp16"))
        self._build_data()
        self.meter = DeviceMeter(self.device)
        self.logger = JsonlLogger(cfg.log_path)
        self.training_acc, self.testing_acc, self.epoch_time = [], [], []
        self.global_step = 0
        self.skipped = torch.zeros((), device=self.device, dtype=torch.int32)  # non-finite steps
        self.profiler = PhaseProfiler(cfg.profile_steps, self.device.type == "cuda", self.logger)
        if cfg.auto_resume and resilience.restore_last(self):
            print0(f"auto-resume: restored {self.last_path}, continuing at epoch {self.start_epoch}")

    # ------------------------------------------------------------------ setup
    @property
    def ckpt_path(self):
        return os.path.join(self.cfg.checkpoint_dir, "resnet_ckpt.pth")

    @property
    def last_path(self):
        return resilience.last_path(self.ckpt_path)

    def _lr(self):
        lr = self.cfg.lr
        if self.cfg.distributed:
            if self.cfg.lr_scaling == "faithful4":
                lr *= 4  # reference hard-codes 4 GPUs (resnet50_test.py:482-485)
            elif self.cfg.lr_scaling == "world":
                lr *= self.world
        return lr

    def _build_optimizer(self):
        cfg = self.cfg
        lr = self._lr()
        kind = cfg.optimizer
        if kind == "auto":
            kind = "ngd" if cfg.ngd else "madgrad"
        if kind == "ngd":
            wd = 1e-4 if cfg.weight_decay is None else cfg.weight_decay
            opt = NGD(self.space, lr=lr, momentum=cfg.momentum, weight_decay=wd)
            if self.zero is not None and self.zero.ws > 1 and "FDT_NGD_GRAPHS" not in os.environ:
                # a rank preconditions ~1/world of the parameters: the step is launch-bound
                # there, and replaying it as HIP graphs wins (world 8 slowest rank, non-update
                # 1.01 -> 0.63 ms, update 3.17 -> 3.01 ms: profiles/r4/ngd_w8_*); at full size
                # (one GPU, world 1 included) the eager step stays the default (GPU-bound:
                # 30.1 vs 30.8 ms unsharded; sharded world 1 30.7 ms with graphs)
                opt.graphs = True
        elif kind == "madgrad":
            wd = 5e-6 if cfg.weight_decay is None else cfg.weight_decay
            opt = MADGRAD(self.space, lr=lr, momentum=cfg.momentum, weight_decay=wd)
        elif kind == "mirror_madgrad":
            wd = 0.0 if cfg.weight_decay is None else cfg.weight_decay
            opt = MirrorMADGRAD(self.space, lr=lr, momentum=cfg.momentum, weight_decay=wd)
        elif kind == "sgd":
            wd = 5e-4 if cfg.weight_decay is None else cfg.weight_decay
            opt = SGD(self.space, lr=lr, momentum=cfg.momentum, weight_decay=wd)
        elif kind in ("adam", "adamw"):
            wd = 0.0 if cfg.weight_decay is None else cfg.weight_decay
            opt = Adam(self.space, lr=lr, weight_decay=wd, adamw=(kind == "adamw"))
        else:
            raise ValueError(kind)
        sched = cfg.scheduler
        if sched == "auto":
            sched = "multistep" if kind == "ngd" else "cosine"
        if sched == "multistep":
            s = torch.optim.lr_scheduler.MultiStepLR(opt, [10, 20], gamma=0.2)
        elif sched == "cosine":
            s = torch.optim.lr_scheduler.CosineAnnealingLR(opt, T_max=200)
        elif sched.startswith("step"):
            gamma = float(cfg.extra.get("gamma", 0.75))
            s = torch.optim.lr_scheduler.StepLR(opt, 2, gamma=gamma)
        elif sched == "none":
            s = None
        else:
            raise ValueError(sched)
        return opt, s

    def _build_data(self):
        cfg = self.cfg
        if cfg.synthetic:
            tr = synthetic_cifar(50000, cfg.num_classes, seed=1)
            te = synthetic_cifar(10000, cfg.num_classes, seed=2)
        else:
            if self.rank == 0:
                CIFAR10(cfg.data_root, train=True, download=True)
            pdist.barrier()
            a, b = CIFAR10(cfg.data_root, train=True), CIFAR10(cfg.data_root, train=False)
            tr, te = (a.data, a.targets), (b.data, b.targets)
        sub = cfg.extra.get("subset_stride")  # tuning: strided 10% subset (C7)
        if sub:
            tr = (tr[0][::sub], tr[1][::sub])
            te = (te[0][::sub], te[1][::sub])
        # Q13: the reference permutes the train transforms once per run; --faithful draws that
        # permutation from the run seed, the default is crop -> flip -> normalise
        self.augment_order = augment_order(cfg.seed, faithful=cfg.faithful)
        self.train_loader = DeviceCIFARLoader(tr[0], tr[1], cfg.bs, self.device, train=True, rank=self.rank,
                                              world_size=self.world, seed=cfg.seed, order=self.augment_order)
        # eval: every rank evaluates the full test set like the reference (no sharding)
        self.test_loader = DeviceCIFARLoader(te[0], te[1], cfg.bs, self.device, train=False, shuffle=False,
                                             drop_last=False)

    # ------------------------------------------------------------------ steps
    def _autocast(self):
        p = self.cfg.precision
        if p == "fp32":
            return torch.autocast(self.device.type, enabled=False)
        dt = torch.bfloat16 if p == "bf16" else torch.float16
        return torch.autocast(self.device.type, dtype=dt, enabled=(self.device.type == "cuda" or p == "bf16"))

    def train_step(self, x, y):
        cfg = self.cfg
        prof = self.profiler
        resilience.maybe_inject_fault(self.global_step, self.rank)
        prof.begin_step()
        if cfg.faithful and self.world > 1:
            # X3: reference DDP (broadcast_buffers=True) re-broadcasts rank 0's BatchNorm
            # running statistics at every forward (resnet50_test.py:716); by default they
            # are synchronised once per epoch and before every evaluation instead
            self._sync_buffers()
        prof.mark("mixup")
        if self.meta is not None:
            x, ya, yb, lam = self.meta(x, y)
        else:
            x, ya, yb, lam = mixup_data(x, y, cfg.alpha)
        prof.mark("forward")
        with self._autocast():
            out = self.model(x)
            prof.mark("loss")
            if self.meta is not None:
                loss = mixup_criterion_meta(None, out, ya, yb, lam, faithful=cfg.faithful, meter=self.meter)
            else:
                loss = mixup_criterion(None, out, ya, yb, lam, meter=self.meter)
        prof.mark("backward")
        if self.scaler.enabled or loss.dtype != torch.float32 or loss.dim() != 0:
            self.scaler.scale_loss(loss).backward()
        else:
            loss.backward(unit_grad(loss.device))
        prof.mark("grad_sync")
        if self.reducer is not None:
            self.reducer.finish()
        if self.sharder is not None:
            self.sharder.finish_backward()
        prof.mark("optimizer")
        fp16 = self.scaler.enabled
        # device-side non-finite check (same kernel as the norm): the optimizer kernels skip
        # the update on a bad step, no host sync (NGD checks on the host: fp16 only)
        guard = cfg.nonfinite_guard and not isinstance(self.optimizer, NGD)
        check = fp16 or guard
        self.clipper(cfg.clip, inv_scale=self.scaler.inv_scale(), check_inf=check)
        found = self.clipper.found_inf if check else None
        if fp16 or (check and self.sharder is not None):
            # fp16 / sharded gradients: every rank must take the same decision
            self.scaler.sync_found_inf(self.clipper.found_inf)
        self.optimizer.step(grad_scale=self.clipper.coef, found_inf=found)
        if fp16:
            self.scaler.update(found)
        if guard:
            self.skipped += found.reshape(())
        if self.sharder is not None:
            self.sharder.after_step()
        self.meter.update(loss, out.detach(), ya, yb, lam.detach() if isinstance(lam, torch.Tensor) else lam)
        prof.end_step()
        self.global_step += 1
        return loss

    def _sync_buffers(self):
        """Rank 0's BatchNorm running statistics to every rank (one collective)."""
        if self.world > 1 and (self.sharder is not None or (self.reducer is not None and self.reducer.broadcast_buffers)):
            pdist.broadcast_buffers(self.model)

    def train_epoch(self, epoch):
        self.model.train()
        self.meter.reset()
        self.train_loader.set_epoch(epoch)  # Q10 fix
        self._sync_buffers()
        if self.device.type == "cuda":
            torch.cuda.synchronize()
            torch.cuda.reset_peak_memory_stats()
        t0 = time.monotonic()
        n = 0
        for i, (x, y) in enumerate(self.train_loader):
            if self.cfg.steps_per_epoch and i >= self.cfg.steps_per_epoch:
                break
            self.train_step(x, y)
            n += 1
        if self.device.type == "cuda":
            torch.cuda.synchronize()
        dt = time.monotonic() - t0
        m = self.meter.reduced()
        imgs = n * self.cfg.bs * self.world
        rec = dict(epoch=epoch, steps=n, epoch_time_s=dt, img_per_s=imgs / max(dt, 1e-9), train_loss=m["loss"],
                   train_acc=m["acc"], peak_mem_gb=peak_memory_gb(), lr=self.optimizer.group["lr"],
                   skipped_steps=int(self.skipped.item()))
        self.skipped.zero_()
        print0(f"epoch {epoch}: {n} steps in {dt:.2f}s ({rec['img_per_s']:.0f} img/s) loss {m['loss']:.4f} "
               f"acc {m['acc']:.2f}%  peak mem {rec['peak_mem_gb']:.2f} GB")
        self.logger.log(**rec)
        self.training_acc.append(m["acc"])
        self.epoch_time.append(dt)
        return rec

    @torch.no_grad()
    def test(self, epoch):
        # every rank evaluates with rank 0's running statistics (reference DDP broadcasts
        # buffers at every forward), so the accuracy -- and the collective "new best ->
        # save" decision below -- is the same on every rank
        self._sync_buffers()
        self.model.eval()
        correct = torch.zeros((), device=self.device)
        total = torch.zeros((), device=self.device)
        loss_sum = torch.zeros((), device=self.device)
        crit = nn.CrossEntropyLoss(reduction="sum")
        for x, y in self.test_loader:
            with self._autocast():
                out = self.model(x)
            loss_sum += crit(out.float(), y)
            correct += (out.argmax(1) == y).sum()
            total += y.numel()
        acc = 100.0 * float(correct) / max(float(total), 1.0)
        acc = pdist.broadcast_scalar(acc)  # one decision for all ranks (save_checkpoint is collective)
        self.testing_acc.append(acc)
        print0(f"test epoch {epoch}: acc {acc:.2f}% loss {float(loss_sum) / max(float(total), 1):.4f}")
        if acc > self.best_acc:
            prefix = self.cfg.distributed or (not self.cfg.distributed and self.cfg.faithful)
            extra = {"optimizer": self.optimizer.state_dict()} if self.cfg.extra.get("save_optimizer") else None
            ckpt.save_checkpoint(self.ckpt_path, self.model, acc, epoch, module_prefix=prefix, extra=extra)
            self.best_acc = acc
        self.logger.log(epoch=epoch, test_acc=acc)
        return acc

    def fit(self):
        for epoch in range(self.start_epoch, self.start_epoch + self.cfg.epoch):
            self.train_epoch(epoch)
            if self.cfg.eval:
                self.test(epoch)
            if self.scheduler is not None:
                self.scheduler.step()
            if self.cfg.save_last or self.cfg.auto_resume:
                resilience.save_last(self, epoch)
        if self.cfg.plot:
            xs = np.arange(self.start_epoch, self.start_epoch + len(self.training_acc))
            if self.testing_acc:
                draw_graph([xs, xs], [self.training_acc, self.testing_acc], ["training", "testing"],
                           "Resnet accuracy curve", "accuracy")
            draw_graph(xs, self.epoch_time, "training time", "Resnet time for training", "time(sec.)")
        return self


def main_ddp(cfg: ResNetConfig):
    t = ResNetTrainer(cfg).fit()
    pdist.cleanup()
    return t
