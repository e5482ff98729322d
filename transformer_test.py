#!/usr/bin/env python3
"""Train the Transformer text classifier on AG News — CLI-compatible with the reference
``transformer_test.py``.

Reference flags (``transformer_test.py:350-361``): --batch_size/-b, --epoch, --lr,
--resume, --workers, --alpha, --distributed, --ngd.  Additional flags: --synthetic,
--seed, --precision, --fsdp, --fsdp_offload, --faithful, --optimizer, --steps, --tokenizer, --data_root,
--layers/--d_model (smaller models for smoke tests), --log, --no_eval, --no_plot.

    python transformer_test.py --synthetic -b 64 --epoch 1
    # the reference's distributed path (transformer_test.py:387-392): FSDP(whole model, CPUOffload)
    torchrun --nproc-per-node 4 transformer_test.py --distributed --faithful --ngd
    bash run_distributed.sh        # torchrun, one rank per GPU
"""
from __future__ import annotations

import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def parse(argv=None):
    p = argparse.ArgumentParser(description="Transformer AG News Training (MI355X engine)")
    p.add_argument("--batch_size", "-b", default=128, type=int)
    p.add_argument("--epoch", default=50, type=int, help="epoch num for training")
    p.add_argument("--lr", default=1e-4, type=float)
    p.add_argument("--resume", action="store_true")
    p.add_argument("--workers", default=2, type=int)
    p.add_argument("--alpha", default=0.99, type=float)
    p.add_argument("--distributed", action="store_true")
    p.add_argument("--ngd", action="store_true")
    # extensions
    p.add_argument("--optimizer", default="auto",
                   choices=["auto", "ngd", "mirror_madgrad", "madgrad", "sgd", "adam", "adamw"])
    p.add_argument("--weight_decay", default=None, type=float)
    p.add_argument("--scheduler", default="onecycle", choices=["onecycle", "multistep"])
    p.add_argument("--synthetic", action="store_true", help="AG-News-shaped synthetic corpus (no download)")
    p.add_argument("--data_root", default="./data")
    p.add_argument("--tokenizer", default="bert-base-uncased",
                   help="HF tokenizer name (local cache) or directory; 'hash' = built-in hash tokenizer (explicit only)")
    p.add_argument("--seed", default=123456, type=int)
    p.add_argument("--precision", default="bf16", choices=["bf16", "fp16", "fp32"])
    p.add_argument("--fsdp", action="store_true", help="flat-sharded data parallel (reference: FSDP)")
    p.add_argument("--fsdp_schedule", default="full_shard", choices=["full_shard", "shard_grad_op"])
    p.add_argument("--fsdp_offload", action="store_true",
                   help="--fsdp: parameter shards in pinned host memory (reference CPUOffload; eager)")
    p.add_argument("--fsdp_offload_optimizer", default="device", choices=["device", "host"],
                   help="--fsdp_offload: optimizer on the GPU over the staged shard (default) or on the host "
                        "(the reference's CPUOffload; --faithful)")
    p.add_argument("--fsdp_wrap", default="model", choices=["model", "sublayer"],
                   help="FSDP units: the whole model (the reference's FSDP(model)) or one per sublayer")
    p.add_argument("--bucket_mb", default=25.0, type=float)
    p.add_argument("--faithful", action="store_true", help="reproduce reference quirks (see README)")
    p.add_argument("--steps", default=0, type=int, help="max steps per epoch (0 = full epoch)")
    p.add_argument("--eval_steps", default=0, type=int)
    p.add_argument("--subset_stride", default=0, type=int, help="strided subset (tuning)")
    p.add_argument("--layers", default=6, type=int)
    p.add_argument("--d_model", default=512, type=int)
    p.add_argument("--no_eval", action="store_true")
    p.add_argument("--no_plot", action="store_true")
    p.add_argument("--checkpoint_dir", default="./checkpoint")
    p.add_argument("--log", default=None)
    p.add_argument("--auto_resume", action="store_true",
                   help="restore <dir>/transformer_last.pth if present (use with torchrun --max-restarts)")
    p.add_argument("--save_last", action="store_true", help="write the full-state transformer_last.pth every epoch")
    p.add_argument("--no_nonfinite_guard", action="store_true")
    p.add_argument("--profile_steps", default=0, type=int, help="per-phase device timing + roctx ranges of K steps")
    return p.parse_args(argv)


def config_from_args(a):
    from faster_distributed_training_amd.train.transformer_trainer import TransformerConfig
    extra = {"scheduler": a.scheduler}
    if a.subset_stride:
        extra["subset_stride"] = a.subset_stride
    if a.eval_steps:
        extra["eval_steps"] = a.eval_steps
    heads = 8 if a.d_model % 8 == 0 else 4
    return TransformerConfig(batch_size=a.batch_size, epoch=a.epoch, lr=a.lr, alpha=a.alpha,
                             distributed=a.distributed, ngd=a.ngd, optimizer=a.optimizer,
                             weight_decay=a.weight_decay, precision=a.precision, synthetic=a.synthetic,
                             data_root=a.data_root, tokenizer=a.tokenizer, seed=a.seed, faithful=a.faithful,
                             fsdp=a.fsdp, fsdp_schedule=a.fsdp_schedule, fsdp_wrap=a.fsdp_wrap, fsdp_offload=a.fsdp_offload, fsdp_offload_optimizer=a.fsdp_offload_optimizer, bucket_mb=a.bucket_mb, resume=a.resume, checkpoint_dir=a.checkpoint_dir,
                             steps_per_epoch=a.steps, eval=not a.no_eval, log_path=a.log, plot=not a.no_plot,
                             workers=a.workers, n_layers=a.layers, d_model=a.d_model, heads=heads,
                             d_ff=2 * a.d_model, d_hidden=2 * a.d_model, auto_resume=a.auto_resume,
                             save_last=a.save_last, nonfinite_guard=not a.no_nonfinite_guard,
                             profile_steps=a.profile_steps, extra=extra)


def main(argv=None):
    a = parse(argv)
    from faster_distributed_training_amd.parallel.dist import cleanup
    from faster_distributed_training_amd.train.transformer_trainer import TransformerTrainer
    trainer = TransformerTrainer(config_from_args(a))
    trainer.fit()
    cleanup()
    return trainer


if __name__ == "__main__":
    main()
