#!/usr/bin/env python3
"""Cost decomposition of the halo 3x3 loop (csrc/kernels/conv_h3.hip) by its probe flags
(ConvArgs.dbg): full kernel, without the LDS-DMA staging (bit 1), without the MFMA phase (bit 2),
without the epilogue (bit 3), and combinations -- device time per call under graph replay.
Outputs are garbage under any flag (timing only).

    python scripts/h3_probe.py --batch 1024
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from faster_distributed_training_amd.ops import _native, conv_igemm as ci  # noqa: E402
from roofline_layers import timeit  # noqa: E402

FLAGS = [(0, "full"), (2, "no DMA"), (4, "no MFMA"), (8, "no epilogue"), (6, "no DMA, no MFMA"),
         (10, "no DMA, no epilogue"), (12, "no MFMA, no epilogue"), (14, "prologue only")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1024)
    a = ap.parse_args()
    dev = torch.device("cuda")
    nat = _native.native()
    N = a.batch
    for H, C in [(32, 64), (16, 128), (8, 256), (4, 512)]:
        shp = ci.ConvShape(C, C, 3, 1, 1)
        x = torch.randn(N, H, H, C, device=dev).to(torch.bfloat16)
        w = torch.randn(C, C, 3, 3, device=dev) / (C * 9) ** 0.5
        wf, wd = ci.alloc_packed(shp, dev)
        ci.pack_weights([(w, wf, wd, shp)])
        part = ci.stat_slots(2, C, dev, N * H * H)
        flop = 2.0 * N * H * H * C * C * 9
        for kg in (6, 7):
            row = []
            for f, name in FLAGS:
                nat.set_conv_debug_flags(f)
                try:
                    t = timeit(lambda: ci.conv_fwd(x, wf, shp, part=part, kg=kg), 20)
                finally:
                    nat.set_conv_debug_flags(0)
                row.append(f"{name} {t * 1e3:6.1f}")
            print(f"N {N} {H}x{H} {C}->{C} fwd kg{kg} ({flop / 1e9:.0f} GFLOP): " + " | ".join(row), flush=True)


if __name__ == "__main__":
    main()
