#!/usr/bin/env python3
"""Run one conv op of one ResNet-50 shape repeatedly (for rocprofv3 --pmc sessions).
    python scripts/prof_layer.py --op fwd --shape 32,64,64,3,1,1 --batch 1024 --tile 128,64,32
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from faster_distributed_training_amd.ops import conv_igemm as ci

ap = argparse.ArgumentParser()
ap.add_argument("--op", default="fwd")
ap.add_argument("--shape", default="32,64,64,3,1,1")
ap.add_argument("--batch", type=int, default=1024)
ap.add_argument("--tile", default=None)
ap.add_argument("--reps", type=int, default=5)
ap.add_argument("--pro", default="affine", choices=["affine", "none"], help="fwd: lazy-BN prologue or a plain operand")
ap.add_argument("--kg", type=int, default=None)
a = ap.parse_args()
H, Cin, Cout, k, s, p = map(int, a.shape.split(","))
tile = tuple(map(int, a.tile.split(","))) if a.tile else None
dev = torch.device("cuda")
N = a.batch
shp = ci.ConvShape(Cin, Cout, k, s, p)
x = torch.randn(N, H, H, shp.cxp, device=dev).to(torch.bfloat16)
w = torch.randn(Cout, Cin, k, k, device=dev) / (Cin * k * k) ** 0.5
wf, wd = ci.alloc_packed(shp, dev)
ci.pack_weights([(w, wf, wd, shp)])
Ho, Wo = ci.out_hw(H, H, shp)
g = torch.randn(N, Ho, Wo, Cout, device=dev).to(torch.bfloat16)
yy = torch.randn(N, Ho, Wo, Cout, device=dev).to(torch.bfloat16)
al = torch.zeros(Cout, device=dev)
be = torch.zeros(Cout, device=dev)
sv = torch.ones(shp.cxp, device=dev)
tv = torch.zeros(shp.cxp, device=dev)
gw = torch.empty(Cout, Cin, k, k, device=dev)
for _ in range(a.reps):
    if a.op == "fwd":
        if a.pro == "none":
            ci.conv_fwd(x, wf, shp, None, None, 0, 1.0, tile=tile, kg=a.kg)
        else:
            ci.conv_fwd(x, wf, shp, sv, tv, 1, 1.0, tile=tile, kg=a.kg)
    elif a.op == "dgrad":
        ci.conv_dgrad(g, yy, al, be, wd, shp, (N, H, H, Cin), tile=tile)
    elif a.op == "wgrad_plain":  # materialised operands (the engine's 3x3 weight gradients); --kg 9: halo
        ci.conv_wgrad(g, None, None, None, x, shp, gw, h3=a.kg == 9)
    else:
        ci.conv_wgrad(g, yy, al, be, x, shp, gw, sv, tv, 1, tile=tile)
torch.cuda.synchronize()
print("ok")
