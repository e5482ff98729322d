#!/usr/bin/env python3
"""Streaming rate of the engine's elementwise passes (residual join, normalise+activate, BN-backward
fold) at the ResNet-50 stage shapes: the one-vector grid-stride form vs the loads-first form
(FDT_EW_UNROLL, bn_kernels.hip kEwU), plus a torch device copy of the same bytes as the
reference rate.  Device time per call (graph replay of 20) and the achieved TB/s."""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from faster_distributed_training_amd.ops import _native  # noqa: E402
from roofline_layers import timeit  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1024)
    a = ap.parse_args()
    dev = torch.device("cuda")
    nat = _native.native()
    sp = _native.stream_ptr
    N = a.batch
    for (H, C) in ((32, 64), (32, 256), (16, 512), (8, 1024), (16, 128), (4, 2048)):
        M = N * H * H
        y = torch.randn(M, C, device=dev).to(torch.bfloat16)
        r = torch.randn(M, C, device=dev).to(torch.bfloat16)
        out = torch.empty_like(y)
        mask = torch.empty(M * C // 8, device=dev, dtype=torch.uint8)
        s, t, s2, t2 = (torch.rand(C, device=dev) + 0.5 for _ in range(4))
        nb = y.numel() * 2
        res = []
        t_copy = timeit(lambda: out.copy_(y), 20) * 1e3
        res.append(f"copy {t_copy:6.1f}us {2 * nb / t_copy / 1e6:4.2f}TB/s")
        for on in (0, 1):
            nat.set_ew_unroll(bool(on))
            t_res = timeit(lambda: nat.residual_act_fwd(y.data_ptr(), s.data_ptr(), t.data_ptr(), r.data_ptr(),
                                                        s2.data_ptr(), t2.data_ptr(), 0, out.data_ptr(),
                                                        mask.data_ptr(), M, C, 1, 1.0, 1, sp()), 20) * 1e3
            t_aa = timeit(lambda: nat.act_affine_fwd(y.data_ptr(), s.data_ptr(), t.data_ptr(), out.data_ptr(), M, C, 1,
                                                     1.0, 1, 1, sp()), 20) * 1e3
            t_af = timeit(lambda: nat.affine_fold(r.data_ptr(), y.data_ptr(), s.data_ptr(), t.data_ptr(), s2.data_ptr(),
                                                  out.data_ptr(), M, C, 1, sp()), 20) * 1e3
            res.append(f"u{on}: join {t_res:6.1f}us {(3 * nb + nb // 16) / t_res / 1e6:4.2f}TB/s  "
                       f"norm {t_aa:6.1f}us {2 * nb / t_aa / 1e6:4.2f}TB/s  fold {t_af:6.1f}us "
                       f"{3 * nb / t_af / 1e6:4.2f}TB/s")
        nat.set_ew_unroll(True)
        # correctness of the streaming form against the one-vector form
        outs = []
        for on in (0, 1):
            nat.set_ew_unroll(bool(on))
            nat.residual_act_fwd(y.data_ptr(), s.data_ptr(), t.data_ptr(), r.data_ptr(), s2.data_ptr(), t2.data_ptr(),
                                 0, out.data_ptr(), mask.data_ptr(), M, C, 1, 1.0, 1, sp())
            o1, m1 = out.clone(), mask.clone()
            nat.act_affine_fwd(y.data_ptr(), s.data_ptr(), t.data_ptr(), out.data_ptr(), M, C, 1, 1.0, 1, 1, sp())
            o2 = out.clone()
            nat.affine_fold(r.data_ptr(), y.data_ptr(), s.data_ptr(), t.data_ptr(), s2.data_ptr(), out.data_ptr(), M, C,
                            1, sp())
            outs.append((o1, m1, o2, out.clone()))
        nat.set_ew_unroll(True)
        same = all(torch.equal(p, q) for p, q in zip(*outs))
        print(f"N {N} {H}x{H}x{C} ({nb / 1e6:.0f} MB per tensor): " + " | ".join(res) + f" | bitwise equal {same}",
              flush=True)
        del y, r, out, mask
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
