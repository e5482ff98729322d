#!/usr/bin/env python3
"""Statistics slot rows vs atomic contention: every ResNet-50 forward convolution shape at a
batch (default 1024) with its shipped tile, timed as conv (stats epilogue) + the fp64 finalize
that sums and re-zeroes the slot rows, for rows in {64, 256, 1024, 4096} (capped at the row
block count).  Device time per (conv + finalize), graph replay of 20."""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from faster_distributed_training_amd.ops import _native  # noqa: E402
from faster_distributed_training_amd.ops import conv_igemm as ci  # noqa: E402
from roofline_layers import timeit  # noqa: E402

SHAPES = [(32, 64, 64, 1), (32, 64, 64, 3), (32, 64, 256, 1), (32, 256, 64, 1),
          (16, 128, 128, 3), (16, 128, 512, 1), (16, 512, 128, 1),
          (8, 256, 256, 3), (8, 256, 1024, 1), (8, 1024, 256, 1),
          (4, 512, 512, 3), (4, 512, 2048, 1), (4, 2048, 512, 1)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--rows", default="64,256,1024,4096")
    a = ap.parse_args()
    dev = torch.device("cuda")
    nat = _native.native()
    rows_list = [int(r) for r in a.rows.split(",")]
    N = a.batch
    for (H, cin, cout, k) in SHAPES:
        shp = ci.ConvShape(cin, cout, k, 1, k // 2)
        x = torch.randn(N, H, H, shp.cxp, device=dev).to(torch.bfloat16)
        w = torch.randn(cout, cin, k, k, device=dev) / (cin * k * k) ** 0.5
        wf, _ = ci.alloc_packed(shp, dev, dgrad=False)
        ci.pack_weights([(w, wf, None, shp)])
        M = N * H * H
        s, t, sm, sa = (torch.empty(cout, device=dev) for _ in range(4))
        res = []
        ref = None
        for R in rows_list:
            if R > max(64, 1 << (-(-M // 64) - 1).bit_length()):
                continue
            part = torch.zeros(R, 2, cout, device=dev)

            def fn():
                ci.conv_fwd(x, wf, shp, part=part)
                nat.stats_finalize(part.data_ptr(), R, cout, float(M), 0, 1e-3, 0.1, 0, 0, 0, 0, 0, s.data_ptr(),
                                   t.data_ptr(), sm.data_ptr(), sa.data_ptr(), 1, _native.stream_ptr())
            us = timeit(fn, 20) * 1e3
            fn()
            torch.cuda.synchronize()
            if ref is None:
                ref = sm.clone()
            err = (sm - ref).abs().max().item()
            res.append(f"R{R} {us:7.1f}us (d {err:.1e})")
        print(f"N {N} {H}x{H} {cin}->{cout} k{k}: " + "  ".join(res), flush=True)


if __name__ == "__main__":
    main()
