#!/usr/bin/env python3
"""Repeatability of the halo 3x3 loop (csrc/kernels/conv_h3.hip): the same launch run many
times must give bitwise-identical outputs and (deterministic mode) statistics -- a missing
barrier between the LDS-DMA fill of a stage and the waves still reading it would show up here
as run-to-run differences.

    python scripts/h3_repeat.py --reps 30
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from faster_distributed_training_amd.ops import _native  # noqa: E402
from faster_distributed_training_amd.ops import conv_igemm as ci  # noqa: E402

SHAPES = [(8, 32, 64, 64), (8, 16, 128, 128), (8, 8, 256, 256), (8, 4, 512, 512), (128, 32, 64, 64),
          (128, 16, 128, 128), (256, 8, 256, 256), (1024, 4, 512, 512)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=30)
    ap.add_argument("--deterministic", type=int, default=1)
    ap.add_argument("--poison", type=int, default=1, help="NaN-fill every CU's LDS before each launch")
    a = ap.parse_args()
    nat = _native.native()
    _native.set_deterministic(bool(a.deterministic))
    dev = torch.device("cuda")
    torch.manual_seed(0)
    bad = 0
    for N, H, C, Co in SHAPES:
        shp = ci.ConvShape(C, Co, 3, 1, 1)
        x = torch.randn(N, H, H, C, device=dev).to(torch.bfloat16)
        w = torch.randn(Co, C, 3, 3, device=dev) / (C * 9) ** 0.5
        wf, wd = ci.alloc_packed(shp, dev)
        ci.pack_weights([(w, wf, wd, shp)])
        g = torch.randn(N, H, H, Co, device=dev).to(torch.bfloat16)
        ex = torch.randn(N, H, H, C, device=dev).to(torch.bfloat16)
        es = torch.rand(C, device=dev) + 0.5
        et = torch.randn(C, device=dev) * 0.3
        M = N * H * H
        for kg in (None, 5, 6, 7, 8):
            for name in ("fwd", "dgrad"):
                if kg == 8 and (Co if name == "fwd" else C) % 128:
                    continue
                outs = []
                sink = torch.zeros(2048 * 256, device=dev, dtype=torch.int32)
                keep = []
                for r in range(a.reps):
                    # a fresh address for every operand copy + (optionally) NaN leftovers in LDS
                    keep.append(torch.empty(4096 * (r + 1), device=dev))
                    if a.poison:
                        nat.lds_poison(sink.data_ptr(), 2048, torch.cuda.current_stream().cuda_stream)
                    if name == "fwd":
                        part = ci.stat_slots(2, Co, dev, M)
                        y, _ = ci.conv_fwd(x, wf, shp, part=part, kg=kg)
                    else:
                        part = ci.stat_slots(2, C, dev, M)
                        y, _ = ci.conv_dgrad(g, None, None, None, wd, shp, (N, H, H, C), epi=ci.EPI_ACTBWD, ex=ex,
                                             es=es, et=et, act=1, part=part, kg=kg)
                    outs.append((y.clone(), part.sum(0)))
                torch.cuda.synchronize()
                nan = sum(int(not (torch.isfinite(o[0].float()).all() and torch.isfinite(o[1]).all())) for o in outs)
                bad += nan
                ny = sum(int(not torch.equal(o[0], outs[0][0])) for o in outs[1:])
                ns = sum(int(not torch.equal(o[1], outs[0][1])) for o in outs[1:])
                bad += ny + ns
                print(f"N {N} {H}x{H} {C}->{Co} {name:5s} kg {kg}: output mismatches {ny}/{a.reps - 1}, "
                      f"statistics mismatches {ns}/{a.reps - 1}, non-finite {nan}", flush=True)
    print("TOTAL mismatches", bad)


if __name__ == "__main__":
    main()
