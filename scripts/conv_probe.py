#!/usr/bin/env python3
"""Where does a small-M convolution's time go?  Device time (graph replay of 20 calls) of one
forward conv as the reduction depth K, the batch (M) and the tile / K-group / loop form vary.

    python scripts/conv_probe.py
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from faster_distributed_training_amd.ops import conv_igemm as ci  # noqa: E402
from roofline_layers import timeit  # noqa: E402


def one(N, H, cin, cout, k, tile, kg=1, ns=1, loop="old"):
    dev = torch.device("cuda")
    shp = ci.ConvShape(cin, cout, k, 1, k // 2)
    x = torch.randn(N, H, H, shp.cxp, device=dev).to(torch.bfloat16)
    w = torch.randn(cout, cin, k, k, device=dev) / (cin * k * k) ** 0.5
    wf, wd = ci.alloc_packed(shp, dev, dgrad=False)
    ci.pack_weights([(w, wf, None, shp)])
    ent = {"tile": list(tile), "nsplit": ns, "kg": kg, "loop": loop}
    orig = ci.tuned
    ci.tuned = lambda op, b, h, s_: ent
    try:
        us = timeit(lambda: ci.conv_fwd(x, wf, shp), 20) * 1e3
    finally:
        ci.tuned = orig
    M = N * H * H
    flop = 2.0 * M * cout * cin * k * k
    nkt = -(-(k * k * shp.cxp) // tile[2])
    return us, flop / us / 1e6, nkt


def main():
    torch.manual_seed(0)
    print("stage-3 3x3 at 8x8, 256 out channels: time vs K (Cin), tile, K groups, loop form")
    for tile, kg in (((64, 128, 64), 1), ((64, 128, 64), 2), ((128, 128, 64), 1), ((64, 64, 64), 1),
                     ((64, 64, 64), 2), ((64, 128, 128), 1)):
        for loop in ("old", "rot") if kg == 1 else ("old",):
            row = []
            for cin in (8, 32, 64, 128, 256, 512):
                us, tf, nkt = one(128, 8, cin, 256, 3, tile, kg=kg, loop=loop)
                row.append(f"Cin {cin:4d} ({nkt:3d} kt) {us:6.1f} us {tf:5.0f} TF")
            print(f"  tile {tile} kg {kg} {loop}: " + " | ".join(row), flush=True)
    print("M sweep (batch), 3x3 256->256 at 8x8, tile 64x128x64 kg 2")
    for N in (32, 64, 128, 256, 512, 1024):
        us, tf, nkt = one(N, 8, 256, 256, 3, (64, 128, 64), kg=2)
        print(f"  N {N:5d}: {us:7.1f} us {tf:5.0f} TF  ({N * 64 // 64 * 2} workgroups)", flush=True)
    print("1x1 1024->256 at 8x8 (M = 8192): time vs tile")
    for tile, kg in (((64, 128, 64), 1), ((64, 128, 64), 2), ((64, 64, 64), 1), ((128, 128, 32), 1)):
        us, tf, nkt = one(128, 8, 1024, 256, 1, tile, kg=kg)
        print(f"  tile {tile} kg {kg}: {us:6.1f} us {tf:5.0f} TF ({nkt} kt)", flush=True)


if __name__ == "__main__":
    main()
