"""Transformer / AG News training driver (reference ``transformer_test.py:152-424``; T3, T4).

Per step (device-resident, no host synchronisation): token batch (packed store, gather +
pad to a length bucket) -> forward with in-model manifold mixup (A5) under bf16 autocast
-> lambda-weighted cross entropy (fused kernel) -> backward (DDP buckets all-reduced
during backward, or flat-sharded FSDP reduce-scatter after it) -> grad-norm clip (10.0)
-> one fused optimizer launch (NGD / MirrorMADGRAD) -> OneCycle LR step.

Reference quirks handled (survey §2.9): Q8 eval crash (tuple output) and mixup active in
eval -> fixed; Q9 OneCycleLR stepped per epoch -> stepped per batch (``faithful`` keeps
per-epoch); Q11 lr x4 -> lr x world (``faithful`` keeps x4); Q17 FSDP + NGD on a flat CPU
shard -> the sharded optimizer owns whole, correctly shaped parameters; Q18 no truncation
-> truncated to maxlen.
"""
from __future__ import annotations

import os
import time
from dataclasses import dataclass, field

import numpy as np
import torch
import torch.nn as nn

from ..data.agnews import NUM_CLASSES, TextBatchLoader, download_agnews, get_tokenizer, load_agnews
from ..models.transformer import Transformer
from ..ops.mixup import mixup_criterion, unit_grad
from ..optim.flat_optim import SGD, Adam, DeviceGradScaler, GradClipper, MirrorMADGRAD, MADGRAD
from ..optim.ngd import NGD
from ..parallel import dist as pdist
from ..ops import _native
from ..parallel.graphs import SegmentedStep, capture_guard as _graph_guard
from ..utils.env import default_device, print0, seed_everything
from ..utils.flat import FlatParams
from . import checkpoint as ckpt
from . import resilience
from .metrics import DeviceMeter, JsonlLogger, PhaseProfiler, draw_graph, peak_memory_gb

TR_GRAPHS = os.environ.get("FDT_TR_GRAPHS", "1") != "0"
# linear / LayerNorm / embedding backward kernels accumulate straight into the flat fp32
# gradient views (ops/linear.py direct gradients) instead of autograd's per-parameter add
DIRECT_GRADS = os.environ.get("FDT_DIRECT_GRADS", "1") != "0"
# bf16 shadow weights kept by the optimizer kernels (utils/flat.py) for the linears
SHADOW = os.environ.get("FDT_TR_SHADOW", "1") != "0"


@dataclass
class TransformerConfig:
    batch_size: int = 128            # per process (reference --batch_size)
    epoch: int = 50
    lr: float = 1e-4
    alpha: float = 0.99              # Beta(alpha, alpha) for manifold mixup
    distributed: bool = False
    ngd: bool = False
    optimizer: str = "auto"          # auto: ngd -> NGD else MirrorMADGRAD (reference)
    weight_decay: float | None = None
    precision: str = "bf16"
    synthetic: bool = False
    data_root: str = "./data"
    tokenizer: str | None = "bert-base-uncased"
    seed: int = 123456
    faithful: bool = False
    fsdp: bool = False
    fsdp_offload: bool = False       # FSDP shards + optimizer state in pinned host memory (reference CPUOffload)
    # where the offloaded run's optimizer runs: "device" = NGD / MADGRAD math + state on the GPU over
    # the staged shard (params still live in pinned host memory between steps), "host" = the
    # reference's CPUOffload optimizer on the CPU (selected by --faithful)
    fsdp_offload_optimizer: str = "device"
    fsdp_param_dtype: str = "fp32"   # fp32 | bf16: all-gather wire / compute copy of the parameters
    fsdp_schedule: str = "full_shard"  # full_shard | shard_grad_op (the HIP-graph path's static FSDP)
    # FSDP wrap units: "model" = the whole model as ONE unit, as the reference wraps it
    # (transformer_test.py:387-392 FSDP(model), no auto-wrap policy): one gather + one
    # reduce-scatter per step -- 12.5 ms/step at batch 256 on one GPU; "sublayer" = embedding /
    # each attention and FFN sublayer / pooler / classifier (gathers prefetched behind compute,
    # ~45 collective actions per step between graph segments, host-bound: 13.8 ms;
    # profiles/r4/tr_fsdp_wrap_*.json)
    fsdp_wrap: str = "model"
    shard_ngd: bool = True           # distributed NGD: each rank owns + preconditions 1/world of the params
    bucket_mb: float = 25.0           # measured faster than 8 MB (profiles/r3s3/ddp_world1_*.json)
    resume: bool = False
    checkpoint_dir: str = "./checkpoint"
    steps_per_epoch: int = 0
    eval: bool = True
    log_path: str | None = None
    plot: bool = True
    workers: int = 2
    n_layers: int = 6
    d_model: int = 512
    heads: int = 8
    d_ff: int = 1024
    d_hidden: int = 1024
    maxlen: int = 512
    length_buckets: tuple = (64, 128, 256, 512)
    clip: float = 10.0
    auto_resume: bool = False        # restore *_last.pth (full state) if present; implies save_last
    save_last: bool = False
    nonfinite_guard: bool = True     # skip (on device) steps whose gradients are not finite
    profile_steps: int = 0
    extra: dict = field(default_factory=dict)


class TransformerTrainer:
    def __init__(self, cfg: TransformerConfig):
        self.cfg = cfg
        self.rank, self.world = 0, 1
        if cfg.distributed or cfg.fsdp or int(os.environ.get("WORLD_SIZE", "1")) > 1:
            # (--fsdp always runs the sharded path, over a world-1 group on one GPU)
            if not torch.distributed.is_initialized():
                pdist.setup_norank()
            self.rank, self.world = pdist.rank(), pdist.world()
            cfg.distributed = self.world > 1
        if cfg.distributed and cfg.faithful and not cfg.fsdp:
            # the reference's --distributed IS FullyShardedDataParallel(model, size_based_auto_wrap_policy,
            # cpu_offload=CPUOffload(offload_params=True)) (transformer_test.py:387-392): at 29.3M
            # parameters the size policy wraps nothing, i.e. ONE unit = the whole model
            cfg.fsdp, cfg.fsdp_wrap, cfg.fsdp_offload = True, "model", True
        self.device = default_device()
        seed_everything(cfg.seed)
        self.tokenizer = get_tokenizer(cfg.tokenizer) if not cfg.synthetic else None
        vocab = self.tokenizer.vocab_size if self.tokenizer is not None else 30522
        self.model = Transformer(NUM_CLASSES, vocab, n_layers=cfg.n_layers, h=cfg.heads, d_model=cfg.d_model,
                                 d_ff=cfg.d_ff, d_hidden=cfg.d_hidden, maxlen=cfg.maxlen, alpha=cfg.alpha,
                                 faithful=cfg.faithful).to(self.device)
        self.best_acc, self.start_epoch = ckpt.load_best_performance(self.ckpt_path, NUM_CLASSES, cfg.resume)
        if cfg.resume:
            ckpt.load_model_state(self.model, ckpt.load_checkpoint(self.ckpt_path)["net"])
        shadow = (SHADOW and self.device.type == "cuda" and cfg.precision == "bf16"
                  and not cfg.fsdp)
        ngd_opt = cfg.optimizer == "ngd" or (cfg.optimizer == "auto" and cfg.ngd)
        self.reducer = self.fsdp = self.zero = None
        if cfg.fsdp:
            # ZeRO-3 (parallel/fsdp.py): parameters sharded at rest, one wrap unit per
            # embedding / attention / FFN sublayer / head, gathered with prefetch and
            # reduce-scattered from gradient hooks; NGD sees whole parameters (Q17)
            from ..parallel.fsdp import FullyShardedDP
            if cfg.fsdp_schedule not in ("full_shard", "shard_grad_op"):
                raise ValueError(f"fsdp_schedule {cfg.fsdp_schedule!r}")
            # static mode (fixed-address unit buffers) when the step will be captured as HIP
            # graphs: each unit's gather / prefetch and reduce-scatter become actions between
            # graph segments (parallel/graphs.SegmentedStep)
            static = bool(self._graphs_wanted() and not cfg.fsdp_offload and cfg.extra.get("fsdp_static", True))
            if cfg.fsdp_wrap not in ("sublayer", "model"):
                raise ValueError(f"fsdp_wrap {cfg.fsdp_wrap!r}")
            self.fsdp = FullyShardedDP(self.model, self.device, mode="param" if ngd_opt else "flat",
                                       units=[("", self.model)] if cfg.fsdp_wrap == "model" else None,
                                       offload=cfg.fsdp_offload, static=static,
                                       offload_optimizer="host" if cfg.faithful else cfg.fsdp_offload_optimizer,
                                       reshard_after_forward=cfg.fsdp_schedule == "full_shard",
                                       param_dtype={"fp32": None, "bf16": torch.bfloat16}[cfg.fsdp_param_dtype])
            self.flat = self.fsdp.space
        else:
            part = self.world if (cfg.distributed and ngd_opt and cfg.shard_ngd) else 0
            # world > 1: per-block Q / K / V adjacency only (whole-model shape runs put
            # every layer's weights in the first buckets -> no all-reduce / backward overlap)
            self.flat = FlatParams(self.model, device=self.device, with_shadow=shadow, partition=part, balance="ngd",
                                   adjacent="layer" if cfg.distributed else "shape")
            if shadow:  # bf16 compute reads the optimizer-maintained bf16 copy (no per-step casts)
                from ..ops.linear import enable_shadow_weights
                enable_shadow_weights(self.flat)
            if part:
                # ZeRO-2 for NGD: every rank preconditions only the parameters it owns
                from ..parallel.zero import ShardedOptimizerDP
                self.zero = ShardedOptimizerDP(self.flat, self.model, bucket_mb=cfg.bucket_mb)
            elif cfg.distributed:
                from ..parallel.ddp import BucketReducer
                self.reducer = BucketReducer(self.flat, self.model, bucket_mb=cfg.bucket_mb)
        self.sharder = self.fsdp if self.fsdp is not None else self.zero
        self.dist_path = self._describe_path(ngd_opt)
        if cfg.distributed or cfg.fsdp:
            print0(f"distributed path: {self.dist_path}")
        if self.fsdp is None and DIRECT_GRADS:
            from ..ops.linear import enable_direct_grads
            enable_direct_grads(self.model.parameters())
        seed_everything(cfg.seed, self.rank)
        self.space = self.sharder.view if self.sharder is not None else self.flat
        self._build_data()
        self.optimizer, self.scheduler = self._build_optimizer()
        self.clipper = GradClipper(self.space, sharded=self.sharder is not None)
        self.scaler = DeviceGradScaler(self.device, enabled=(cfg.precision == "fp16"))
        self.meter = DeviceMeter(self.device)
        self.logger = JsonlLogger(cfg.log_path)
        self.pos_index = torch.arange(cfg.maxlen, device=self.device)  # transformer_test.py:228
        self.training_acc, self.testing_acc, self.epoch_time = [], [], []
        self.global_step = 0
        self.skipped = torch.zeros((), device=self.device, dtype=torch.int32)
        self.profiler = PhaseProfiler(cfg.profile_steps, self.device.type == "cuda", self.logger)
        self._graphs, self._graph_stream, self._graph_pool = {}, None, None
        if cfg.auto_resume and resilience.restore_last(self):
            print0(f"auto-resume: restored {self.last_path}, continuing at epoch {self.start_epoch}")

    def _describe_path(self, ngd_opt):
        """Which data-parallel path this run takes (printed at start; the reference's
        --distributed is FSDP(model) + CPU offload, ``--faithful`` selects exactly that)."""
        cfg = self.cfg
        if self.fsdp is not None:
            wrap = "whole model as one unit" if cfg.fsdp_wrap == "model" else "one unit per sublayer"
            mode = "static, HIP-graph segments" if self.fsdp.static else "eager"
            off = ((", CPU offload (host optimizer)" if (cfg.faithful or cfg.fsdp_offload_optimizer == "host")
                    else ", CPU offload (device optimizer)") if cfg.fsdp_offload else "")
            ref = " -- the reference's FSDP(model, CPUOffload)" if (cfg.fsdp_offload and cfg.fsdp_wrap == "model") else ""
            return f"FSDP {cfg.fsdp_schedule} ({wrap}, {mode}{off}), world {self.world}{ref}"
        if self.zero is not None:
            return f"DDP buckets + ZeRO-2 sharded NGD, world {self.world} (reference: FSDP + CPU offload; --faithful)"
        if self.reducer is not None:
            return f"DDP bucket reducer, world {self.world} (reference: FSDP + CPU offload; --faithful)"
        return "single process"

    @property
    def ckpt_path(self):
        return os.path.join(self.cfg.checkpoint_dir, "transformer_ckpt.pth")

    @property
    def last_path(self):
        return resilience.last_path(self.ckpt_path)

    def _build_data(self):
        cfg = self.cfg
        if not cfg.synthetic:
            # one rank downloads (reference: AG_NEWS(root='./data'), transformer_test.py:88-93);
            # everyone then reads, and fails the same way if the data is still missing
            if self.rank == 0:
                try:
                    download_agnews(cfg.data_root)
                except Exception as e:  # noqa: BLE001 - reported by load_agnews below on every rank
                    print(f"AG News download failed: {type(e).__name__}: {e}", flush=True)
            from ..parallel.dist import barrier
            barrier()
        tr = load_agnews(cfg.data_root, True, self.tokenizer, cfg.maxlen, cfg.synthetic, seed=1, download=False)
        te = load_agnews(cfg.data_root, False, self.tokenizer, cfg.maxlen, cfg.synthetic, seed=1, download=False)
        sub = cfg.extra.get("subset_stride")
        if sub:
            from ..data.agnews import TokenStore
            tr = TokenStore([tr.sample(i)[0] for i in range(0, len(tr), sub)], tr.labels[::sub])
            te = TokenStore([te.sample(i)[0] for i in range(0, len(te), sub)], te.labels[::sub])
        self.train_loader = TextBatchLoader(tr, cfg.batch_size, self.device, rank=self.rank, world_size=self.world,
                                            seed=cfg.seed, length_buckets=cfg.length_buckets)
        # eval: every rank evaluates the full test set, as the reference does
        self.test_loader = TextBatchLoader(te, cfg.batch_size, self.device, shuffle=False, drop_last=False,
                                           length_buckets=cfg.length_buckets)

    def _lr(self):
        lr = self.cfg.lr
        if self.cfg.distributed:
            lr *= 4 if self.cfg.faithful else self.world  # reference hard-codes 4 (Q11)
        return lr

    def _build_optimizer(self):
        cfg = self.cfg
        lr = self._lr()
        kind = cfg.optimizer
        if kind == "auto":
            kind = "ngd" if cfg.ngd else "mirror_madgrad"
        wd = cfg.weight_decay
        if kind == "ngd":
            opt = NGD(self.space, lr=lr, weight_decay=wd or 0.0)
            if self.zero is not None and self.zero.ws > 1 and "FDT_NGD_GRAPHS" not in os.environ:
                # as the ResNet trainer (resnet_trainer.py _build_optimizer): a rank preconditions
                # ~1/world of the parameters, so its NGD step is launch-bound and replays as HIP
                # graphs; the full-size step (one GPU) stays eager (GPU-bound)
                opt.graphs = True
        elif kind == "mirror_madgrad":
            opt = MirrorMADGRAD(self.space, lr=lr, momentum=0.9, weight_decay=wd or 0.0)
        elif kind == "madgrad":
            opt = MADGRAD(self.space, lr=lr, momentum=0.9, weight_decay=wd or 0.0)
        elif kind == "sgd":
            opt = SGD(self.space, lr=lr, momentum=0.0, weight_decay=wd or 0.0)
        elif kind in ("adam", "adamw"):
            opt = Adam(self.space, lr=lr, weight_decay=wd or 0.0, adamw=kind == "adamw")
        else:
            raise ValueError(kind)
        steps = self.cfg.steps_per_epoch or len(self.train_loader)
        if cfg.extra.get("scheduler") == "multistep":  # tuning variant (tuning/transformer_tuning.py:204)
            sch = torch.optim.lr_scheduler.MultiStepLR(opt, [10, 15], gamma=0.1)
        else:
            sch = torch.optim.lr_scheduler.OneCycleLR(opt, max_lr=5 * lr, epochs=cfg.epoch,
                                                      steps_per_epoch=max(1, steps), cycle_momentum=True)
        return opt, sch

    def _autocast(self, cache=True):
        p = self.cfg.precision
        if p == "fp32":
            return torch.autocast(self.device.type, enabled=False)
        dt = torch.bfloat16 if p == "bf16" else torch.float16
        return torch.autocast(self.device.type, dtype=dt, enabled=(self.device.type == "cuda" or p == "bf16"),
                              cache_enabled=cache)

    # ------------------------------------------------------------ HIP graphs
    # The transformer step is ~700 kernels, many of them short: the host, not the GPU,
    # bounds it (measured: 4.1 ms of a 16.8 ms step idle between kernels).  Forward, loss
    # and backward of one batch shape are captured once into a HIP graph and replayed;
    # per-step randomness stays live: the manifold-mixup permutation and lambda are written
    # into static device buffers before each replay, torch's dropout advances its philox
    # offset per replay, and the attention kernels XOR a per-replay device seed into their
    # dropout hash (ops/attention_native.py DEVICE_SEED).  Gradients accumulate into the
    # flat gradient buffer (static; the optimizer zeroes it).  Under DDP the capture is cut
    # where a gradient bucket completes (parallel/graphs.SegmentedStep) and the replay
    # launches each bucket's all-reduce between segments (also under the sharded NGD
    # optimizer, whose gradient all-reduce is the same bucket reducer).  Under static FSDP the
    # forward is cut at every unit too (gather wait + prefetch between segments).  bf16 only.
    def _graphs_wanted(self):
        # (the --no-native ablation is plain eager PyTorch by default: graphs are one of the
        # "tricks".  ``extra["graphs_torch_ops"]`` captures the torch-op step too -- graph-safe
        # since its embedding backward is a static-shape index_add (ops/embedding._GatherRows;
        # ATen's dense embedding backward sized its unique/partition buffers at capture time
        # and faulted on replay), with parallel.graphs.capture_guard refusing any such op)
        from ..ops import _native
        cfg = self.cfg
        native_ok = _native.enabled() or bool(cfg.extra.get("graphs_torch_ops"))
        return (TR_GRAPHS and self.device.type == "cuda" and native_ok and cfg.precision != "fp16"
                and cfg.profile_steps <= 0 and not cfg.faithful)

    def _graphs_on(self):
        # under FSDP only the static (fixed-address) mode can be captured
        return (self._graphs_wanted() and (self.fsdp is None or self.fsdp.static) and not self.scaler.enabled
                and self.model.training)

    def _fwd_bwd(self, tokens, labels, types, masks):
        prof = self.profiler
        mask = masks.view(masks.shape[0], 1, 1, masks.shape[1])
        with self._autocast():
            logits, perm, lam = self.model(tokens, types, self.pos_index, mask)
            prof.mark("loss")
            loss = mixup_criterion(None, logits, labels, labels[perm], lam, meter=self.meter)
        prof.mark("backward")
        if self.scaler.enabled or loss.dtype != torch.float32 or loss.dim() != 0:
            self.scaler.scale_loss(loss).backward()
        else:
            loss.backward(unit_grad(loss.device))  # (no seed fill, no d(logits) scaling pass)
        return loss, logits, perm, lam

    def _graph_fill(self, st, tokens, labels, types, masks):
        st["tokens"].copy_(tokens, non_blocking=True)
        st["types"].copy_(types, non_blocking=True)
        st["masks"].copy_(masks, non_blocking=True)
        st["labels"].copy_(labels, non_blocking=True)
        lam = self.model.sample_lam()
        if st.get("prep"):
            # one kernel (csrc/kernels/mixup.hip mixup_prep): the device permutation seeded from
            # the host generator, the permuted labels and the lambda vector -- instead of
            # randperm's sort passes, a label gather and a fill
            seed = int(torch.randint(0, 2**62, (1,)).item())
            _native.native().mixup_prep(st["labels"].data_ptr(), st["labels"].shape[0], float(lam), seed,
                                        st["perm"].data_ptr(), st["yb"].data_ptr(), st["lam"].data_ptr(),
                                        _native.stream_ptr())
        else:
            torch.randperm(tokens.shape[0], device=self.device, out=st["perm"])
            st["lam"].fill_(lam)
        st["seed"].random_()
        return lam

    def _fwd_bwd_graphed(self, tokens, labels, types, masks):
        from ..ops import attention_native as AN
        from ..ops.mixup import mixup_cross_entropy
        key = (tuple(tokens.shape), tuple(masks.shape), str(tokens.dtype))
        ent = self._graphs.get(key, 0)
        if isinstance(ent, int):
            if self._graph_stream is None:
                self._graph_stream = torch.cuda.Stream(device=self.device)
                self._graph_pool = torch.cuda.graph_pool_handle()
            if ent < 2:  # eager warm-up steps on a side stream (lazy library / allocator init)
                self._graphs[key] = ent + 1
                s = self._graph_stream
                s.wait_stream(torch.cuda.current_stream())
                with torch.cuda.stream(s):
                    out = self._fwd_bwd(tokens, labels, types, masks)
                torch.cuda.current_stream().wait_stream(s)
                return out
            B = tokens.shape[0]
            prep = (labels.dtype == torch.int64 and 1 <= B <= 1024 and hasattr(_native.native(), "mixup_prep")
                    and os.environ.get("FDT_TR_MIXUP_PREP", "1") != "0")
            st = dict(tokens=torch.empty_like(tokens), types=torch.empty_like(types), masks=torch.empty_like(masks),
                      labels=torch.empty_like(labels),
                      perm=torch.empty(B, dtype=torch.int32 if prep else torch.long, device=self.device),
                      yb=torch.empty_like(labels),
                      lam=torch.empty(B, dtype=torch.float32, device=self.device),
                      seed=torch.zeros(1, dtype=torch.int64, device=self.device), prep=prep)
            def fwd():
                mask = st["masks"].view(B, 1, 1, st["masks"].shape[1])
                with self._autocast(cache=False):  # no cast cache across a graph capture
                    logits, perm, _ = self.model(st["tokens"], st["types"], self.pos_index, mask)
                    yb = st["yb"] if prep else st["labels"][perm]
                    # the loss kernel also accumulates the step's loss / accuracy into the meter
                    # (captured: every replay adds; DeviceMeter.reset zeroes in place)
                    loss = mixup_cross_entropy(logits, st["labels"], yb, st["lam"],
                                               meter=self.meter if os.environ.get("FDT_TR_GRAPH_METER", "1") != "0"
                                               else None)
                return loss, logits

            torch.cuda.synchronize()
            AN.DEVICE_SEED = st["seed"]
            self.model.mix_override = (st["perm"], st["lam"])
            try:
                if self.reducer is not None or self.zero is not None or self.fsdp is not None:
                    # bucket all-reduces / FSDP reduce-scatters gated on event nodes of the
                    # backward graph (or launched between segments), FSDP gathers between the
                    # forward's segments
                    step = SegmentedStep(self.device, self._graph_pool, stream=self._graph_stream)
                    loss, logits = step.capture(fwd)
                    st.update(replay=step.replay, segments=step.num_segments, step=step)
                else:
                    g = torch.cuda.CUDAGraph()
                    with torch.cuda.graph(g, pool=self._graph_pool), _graph_guard():
                        loss, logits = fwd()
                        loss.backward(unit_grad(loss.device))
                    st.update(replay=g.replay, segments=1)
            finally:
                AN.DEVICE_SEED = None
                self.model.mix_override = None
            st.update(loss=loss, logits=logits, meter=bool(self.meter.fused))
            self.meter.fused = False
            self._graphs[key] = ent = st
        lam = self._graph_fill(ent, tokens, labels, types, masks)
        ent["replay"]()
        if ent["meter"]:
            self.meter.fused = True  # this replay accumulated the meter (train_step: count only)
        step = ent.get("step")
        if step is not None and step.rec.needs_check:
            # first replay with the bucket all-reduces captured in-graph: checked against eager
            # all-reduces (parallel/graphs.py); the next step recaptures without the snapshots
            # (capture mode stands) or with cuts (fallback)
            step.rec.check_collectives()
            self._graphs[key] = 2
            # the checking step's graphs are dropped here: their private pool's use count falls to
            # zero, and a capture into a pool in that state trips the caching allocator's assert
            # (found by the world-8 rehearsal, bench.py --simulate-world 8): recapture into a new pool
            self._graph_pool = torch.cuda.graph_pool_handle()
        return ent["loss"], ent["logits"], ent["perm"], lam

    def train_step(self, tokens, labels, types, masks):
        cfg = self.cfg
        prof = self.profiler
        resilience.maybe_inject_fault(self.global_step, self.rank)
        prof.begin_step()
        prof.mark("forward")
        if self._graphs_on():
            loss, logits, perm, lam = self._fwd_bwd_graphed(tokens, labels, types, masks)
        else:
            loss, logits, perm, lam = self._fwd_bwd(tokens, labels, types, masks)
        prof.mark("grad_sync")
        if self.reducer is not None:
            self.reducer.finish()
        if self.sharder is not None:
            self.sharder.finish_backward()
        prof.mark("optimizer")
        fp16 = self.scaler.enabled
        guard = cfg.nonfinite_guard and not isinstance(self.optimizer, NGD)  # NGD: host check, fp16 only
        check = fp16 or guard
        self.clipper(cfg.clip, inv_scale=self.scaler.inv_scale(), check_inf=check)
        found = self.clipper.found_inf if check else None
        if fp16 or (check and self.sharder is not None):
            self.scaler.sync_found_inf(self.clipper.found_inf)
        self.optimizer.step(grad_scale=self.clipper.coef, found_inf=found)
        if fp16:
            self.scaler.update(found)
        if guard:
            self.skipped += found.reshape(())
        if self.sharder is not None:
            self.sharder.after_step()
        if not cfg.faithful and self.scheduler is not None and isinstance(
                self.scheduler, torch.optim.lr_scheduler.OneCycleLR):
            if self.scheduler.last_epoch + 1 < self.scheduler.total_steps:
                self.scheduler.step()  # per batch, as OneCycleLR intends (Q9)
        self.meter.update(loss, logits.detach(), labels, None if self.meter.fused else labels[perm.long()], lam)
        prof.end_step()
        self.global_step += 1
        return loss

    def train_epoch(self, epoch):
        self.model.train()
        self.meter.reset()
        self.train_loader.set_epoch(epoch)
        if self.device.type == "cuda":
            torch.cuda.synchronize()
            torch.cuda.reset_peak_memory_stats()
        t0 = time.monotonic()
        n = 0
        for i, batch in enumerate(self.train_loader):
            if self.cfg.steps_per_epoch and i >= self.cfg.steps_per_epoch:
                break
            self.train_step(*batch)
            n += 1
        if self.device.type == "cuda":
            torch.cuda.synchronize()
        dt = time.monotonic() - t0
        m = self.meter.reduced()
        samples = n * self.cfg.batch_size * self.world
        rec = dict(epoch=epoch, steps=n, epoch_time_s=dt, samples_per_s=samples / max(dt, 1e-9), train_loss=m["loss"],
                   train_acc=m["acc"], peak_mem_gb=peak_memory_gb(), lr=self.optimizer.group["lr"],
                   skipped_steps=int(self.skipped.item()))
        self.skipped.zero_()
        print0(f"epoch {epoch}: {n} steps in {dt:.2f}s ({rec['samples_per_s']:.0f} samples/s) loss {m['loss']:.4f} "
               f"acc {m['acc']:.2f}%  peak mem {rec['peak_mem_gb']:.2f} GB")
        self.logger.log(**rec)
        self.training_acc.append(m["acc"])
        self.epoch_time.append(dt)
        return rec

    @torch.no_grad()
    def test(self, epoch):
        """Reference ``test`` (``transformer_test.py:300-347``) with Q8 fixed: no mixup in
        eval and the logits are taken from the returned tuple."""
        self.model.eval()
        correct = torch.zeros((), device=self.device)
        total = torch.zeros((), device=self.device)
        for i, (tokens, labels, types, masks) in enumerate(self.test_loader):
            if self.cfg.extra.get("eval_steps") and i >= self.cfg.extra["eval_steps"]:
                break
            with self._autocast():
                logits, _, _ = self.model(tokens, types, self.pos_index, masks.view(masks.shape[0], 1, 1, -1))
            correct += (logits.argmax(1) == labels).sum()
            total += labels.numel()
        acc = 100.0 * float(correct) / max(float(total), 1.0)
        acc = pdist.broadcast_scalar(acc)  # one decision for all ranks (save_checkpoint is collective)
        self.testing_acc.append(acc)
        print0(f"test epoch {epoch}: acc {acc:.2f}%")
        if acc > self.best_acc:
            ckpt.save_checkpoint(self.ckpt_path, self.model, acc, epoch, module_prefix=self.cfg.distributed)
            self.best_acc = acc
        self.logger.log(epoch=epoch, test_acc=acc)
        return acc

    def fit(self):
        for epoch in range(self.start_epoch, self.start_epoch + self.cfg.epoch):
            self.train_epoch(epoch)
            if self.cfg.faithful and self.scheduler is not None:
                self.scheduler.step()  # reference: once per epoch (transformer_test.py:291)
            elif not isinstance(self.scheduler, torch.optim.lr_scheduler.OneCycleLR) and self.scheduler is not None:
                self.scheduler.step()
            if self.cfg.eval:
                self.test(epoch)
            if self.cfg.save_last or self.cfg.auto_resume:
                resilience.save_last(self, epoch)
        if self.cfg.plot:
            xs = np.arange(self.start_epoch, self.start_epoch + len(self.training_acc))
            if self.testing_acc:
                draw_graph([xs, xs], [self.training_acc, self.testing_acc], ["training", "testing"],
                           "Transformer accuracy curve", "accuracy")
            draw_graph(xs, self.epoch_time, "training time", "Transformer time for training", "time(sec.)")
        return self
