#!/usr/bin/env python3
"""Train ResNet on CIFAR-10 — CLI-compatible with the reference ``resnet50_test.py``.

Reference flags (``resnet50_test.py:46-59``): --lr, --resume/-r, --epoch, --alpha, --bs,
--workers, --meta_learning, --distributed, --ngd.  Additional flags: --synthetic,
--seed, --precision, --fsdp, --fsdp_offload, --bucket_mb, --faithful, --optimizer, --arch, --steps,
--weight_decay/--gamma (tuning variant), --data_root, --log, --no_eval.

Examples (single MI355X, or via torchrun / run_distributed.sh for several):
    python resnet50_test.py --bs 64 --ngd --meta_learning
    python resnet50_test.py --bs 1024 --synthetic --epoch 1
"""
from __future__ import annotations

import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def parse(argv=None):
    p = argparse.ArgumentParser(description="PyTorch CIFAR10 Training (MI355X engine)")
    p.add_argument("--lr", default=0.02, type=float, help="learning rate")
    p.add_argument("--resume", "-r", action="store_true", help="resume from checkpoint")
    p.add_argument("--epoch", default=50, type=int, help="epoch num for training")
    p.add_argument("--alpha", default=0.99, type=float, help="alpha value for beta distribution")
    p.add_argument("--bs", default=128, type=int)
    p.add_argument("--workers", default=2, type=int)
    p.add_argument("--meta_learning", action="store_true", help="adaptive lambda in mixup")
    p.add_argument("--distributed", action="store_true")
    p.add_argument("--ngd", action="store_true")
    # extensions
    p.add_argument("--arch", default="resnet50", choices=["resnet18", "resnet34", "resnet50", "resnet101", "resnet152"])
    p.add_argument("--optimizer", default="auto", choices=["auto", "ngd", "madgrad", "mirror_madgrad", "sgd", "adam", "adamw"])
    p.add_argument("--weight_decay", default=None, type=float)
    p.add_argument("--gamma", default=None, type=float, help="StepLR gamma (tuning variant)")
    p.add_argument("--scheduler", default="auto")
    p.add_argument("--synthetic", action="store_true", help="CIFAR-shaped synthetic data (no download)")
    p.add_argument("--data_root", default="./data")
    p.add_argument("--seed", default=123456, type=int)
    p.add_argument("--precision", default="bf16", choices=["bf16", "fp16", "fp32"])
    p.add_argument("--fsdp", action="store_true")
    p.add_argument("--fsdp_schedule", default="full_shard", choices=["full_shard", "shard_grad_op"])
    p.add_argument("--fsdp_offload", action="store_true",
                   help="--fsdp: parameter shards in pinned host memory (reference CPUOffload; eager)")
    p.add_argument("--fsdp_offload_optimizer", default="device", choices=["device", "host"],
                   help="--fsdp_offload: optimizer on the GPU over the staged shard (default) or on the host "
                        "(the reference's CPUOffload; --faithful)")
    p.add_argument("--bucket_mb", default=25.0, type=float)
    p.add_argument("--comm_dtype", default="fp32", choices=["fp32", "bf16"])
    p.add_argument("--faithful", action="store_true", help="reproduce reference quirks (lr x4, mixup loss form)")
    p.add_argument("--learnable_meta", action="store_true", help="optimise the meta-mixup lambda")
    p.add_argument("--steps", default=0, type=int, help="max steps per epoch (0 = full epoch)")
    p.add_argument("--subset_stride", default=0, type=int, help="train/test on a strided subset (tuning)")
    p.add_argument("--no_eval", action="store_true")
    p.add_argument("--no_plot", action="store_true")
    p.add_argument("--checkpoint_dir", default="./checkpoint")
    p.add_argument("--log", default=None, help="JSONL metrics path")
    p.add_argument("--auto_resume", action="store_true",
                   help="restore the full-state checkpoint <dir>/resnet_last.pth if present (use with torchrun --max-restarts)")
    p.add_argument("--save_last", action="store_true", help="write the full-state resnet_last.pth every epoch")
    p.add_argument("--no_nonfinite_guard", action="store_true", help="do not skip steps with non-finite gradients")
    p.add_argument("--profile_steps", default=0, type=int, help="per-phase device timing + roctx ranges of K steps")
    p.add_argument("--no_graphs", action="store_true", help="launch the engine's kernels eagerly (no HIP graphs)")
    p.add_argument("--deterministic", action="store_true",
                   help="bitwise-repeatable engine steps: ordered statistics/split-K reductions, no shared fp32 atomics")
    return p.parse_args(argv)


def config_from_args(a):
    from faster_distributed_training_amd.train.resnet_trainer import ResNetConfig
    extra = {}
    if a.gamma is not None:
        extra["gamma"] = a.gamma
    if a.subset_stride:
        extra["subset_stride"] = a.subset_stride
    sched = a.scheduler
    if a.gamma is not None and sched == "auto":
        sched = "step"
    return ResNetConfig(arch=a.arch, bs=a.bs, lr=a.lr, epoch=a.epoch, alpha=a.alpha, meta_learning=a.meta_learning,
                        learnable_meta=a.learnable_meta, distributed=a.distributed, ngd=a.ngd,
                        optimizer=a.optimizer, weight_decay=a.weight_decay, precision=a.precision,
                        synthetic=a.synthetic, data_root=a.data_root, seed=a.seed, faithful=a.faithful,
                        lr_scaling="faithful4" if a.faithful else "world", bucket_mb=a.bucket_mb,
                        comm_dtype=a.comm_dtype, fsdp=a.fsdp, fsdp_schedule=a.fsdp_schedule, fsdp_offload=a.fsdp_offload, fsdp_offload_optimizer=a.fsdp_offload_optimizer, scheduler=sched, resume=a.resume,
                        checkpoint_dir=a.checkpoint_dir, steps_per_epoch=a.steps, eval=not a.no_eval,
                        log_path=a.log, plot=not a.no_plot, workers=a.workers, auto_resume=a.auto_resume,
                        save_last=a.save_last, nonfinite_guard=not a.no_nonfinite_guard,
                        profile_steps=a.profile_steps, graphs=not a.no_graphs,
                        deterministic=a.deterministic, extra=extra)


def main(argv=None):
    a = parse(argv)
    from faster_distributed_training_amd.parallel.dist import cleanup
    from faster_distributed_training_amd.train.resnet_trainer import ResNetTrainer
    trainer = ResNetTrainer(config_from_args(a))
    trainer.fit()
    cleanup()
    return trainer


if __name__ == "__main__":
    main()
