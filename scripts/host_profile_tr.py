#!/usr/bin/env python3
"""Host-side profile (cProfile) of the Transformer training step at a given batch: where the
Python / launch time of a step goes once the device work is graph-replayed."""
import argparse
import cProfile
import os
import pstats
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--steps", type=int, default=20)
    a = ap.parse_args()
    from faster_distributed_training_amd.train.transformer_trainer import TransformerConfig, TransformerTrainer
    tr = TransformerTrainer(TransformerConfig(batch_size=a.batch, synthetic=True, eval=False, plot=False, ngd=True,
                                              length_buckets=(128, 256), epoch=1))
    it = iter(tr.train_loader)
    tr.model.train()
    for _ in range(14):
        tr.train_step(*next(it))
    torch.cuda.synchronize()
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(a.steps):
        tr.train_step(*next(it))
    torch.cuda.synchronize()
    pr.disable()
    st = pstats.Stats(pr)
    st.sort_stats("cumulative").print_stats(45)
    st.sort_stats("tottime").print_stats(30)


if __name__ == "__main__":
    main()
