#!/usr/bin/env python3
"""Which tuned-table entries (op key, shape key) and launch configs one engine training step
actually uses -- to check that scripts/retune_graph.py tuned the calls the engine makes.

    python scripts/engine_launch_keys.py --batch 1024
"""
import argparse
import collections
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from faster_distributed_training_amd.ops import conv_igemm as ci  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1024)
    a = ap.parse_args()
    from faster_distributed_training_amd.train.resnet_trainer import ResNetConfig, ResNetTrainer
    tr = ResNetTrainer(ResNetConfig(arch="resnet50", bs=a.batch, synthetic=True, eval=False, plot=False,
                                    graphs=False))
    orig = ci.tuned
    seen = collections.Counter()

    def spy(op, batch, h, shp):
        e = orig(op, batch, h, shp)
        seen[(op, ci.tune_key(batch, h, shp), bool(e))] += 1
        return e
    ci.tuned = spy
    ci.LAUNCH_LOG = []
    it = iter(tr.train_loader)
    tr.model.train()
    tr.train_step(*next(it))
    torch.cuda.synchronize()
    for (op, key, hit), n in sorted(seen.items(), key=lambda kv: (kv[0][1], kv[0][0])):
        print(f"{key:24s} {op:9s} {'hit ' if hit else 'MISS'} x{n}")
    launches = collections.Counter(ci.LAUNCH_LOG)
    print("launches:")
    for (kind, key, hit, tile, ns, kg), n in sorted(launches.items(), key=lambda kv: kv[0][1]):
        print(f"  {kind:8s} {key:24s} tuned={hit} tile={tile} ns={ns} kg={kg} x{n}")


if __name__ == "__main__":
    main()
