#!/usr/bin/env python3
"""Residual join + the next block's first 1x1 conv: standalone join pass (residual_act_fwd)
followed by the conv of its output, vs the join folded into the conv's operand staging
(conv_fwd_join) at several tiles.  Device time per pair (graph replay of 20)."""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from faster_distributed_training_amd.ops import _native  # noqa: E402
from faster_distributed_training_amd.ops import conv_igemm as ci  # noqa: E402
from roofline_layers import timeit  # noqa: E402

# (H, block width C4 = join channels, next conv's output channels)
SHAPES = [(32, 256, 64), (16, 512, 128), (8, 1024, 256), (4, 2048, 512)]
TILES = [(256, 128, 32), (128, 128, 64), (128, 64, 64), (64, 128, 64), (64, 64, 64), (64, 256, 64), (128, 256, 32),
         (128, 256, 64)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1024)
    a = ap.parse_args()
    dev = torch.device("cuda")
    nat = _native.native()
    N = a.batch
    for (H, C, cout) in SHAPES:
        shp = ci.ConvShape(C, cout, 1, 1, 0)
        M = N * H * H
        y = torch.randn(N, H, H, C, device=dev).to(torch.bfloat16)
        r = torch.randn(N, H, H, C, device=dev).to(torch.bfloat16)
        s, t, s2, t2 = (torch.rand(C, device=dev) + 0.5 for _ in range(4))
        out = torch.empty_like(y)
        mask = torch.empty(M * C // 8, device=dev, dtype=torch.uint8)
        w = torch.randn(cout, C, 1, 1, device=dev) / C ** 0.5
        wf, _ = ci.alloc_packed(shp, dev, dgrad=False)
        ci.pack_weights([(w, wf, None, shp)])
        part = ci.stat_slots(2, cout, dev, M)

        def sep():
            nat.residual_act_fwd(y.data_ptr(), s.data_ptr(), t.data_ptr(), r.data_ptr(), s2.data_ptr(), t2.data_ptr(),
                                 0, out.data_ptr(), mask.data_ptr(), M, C, 1, 1.0, 1, _native.stream_ptr())
            return ci.conv_fwd(out, wf, shp, part=part)[0]
        t_join = timeit(lambda: nat.residual_act_fwd(y.data_ptr(), s.data_ptr(), t.data_ptr(), r.data_ptr(),
                                                     s2.data_ptr(), t2.data_ptr(), 0, out.data_ptr(), mask.data_ptr(),
                                                     M, C, 1, 1.0, 1, _native.stream_ptr()), 20) * 1e3
        t_sep = timeit(sep, 20) * 1e3
        ref = sep().float()
        ref_out = out.clone()
        res = [f"join {t_join:6.1f} + conv = {t_sep:6.1f} us"]
        for tile in TILES:
            if cout % tile[1]:
                continue
            out.zero_()
            fn = lambda: ci.conv_fwd_join(y, r, s, t, s2, t2, wf, shp, out, mask, part=part, tile=tile)[0]  # noqa: E731
            us = timeit(fn, 20) * 1e3
            o = fn().float()
            err = (o - ref).abs().max().item()
            eo = (out.float() - ref_out.float()).abs().max().item()
            res.append(f"{tile}: {us:6.1f} (d {err:.1e}/{eo:.1e})")
        print(f"N {N} {H}x{H} join {C} -> conv {C}->{cout}: " + "  ".join(res), flush=True)


if __name__ == "__main__":
    main()
