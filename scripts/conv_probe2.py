#!/usr/bin/env python3
"""Fixed cost of a convolution launch at the 8-GPU per-GPU batch: statistics epilogue (fp32
atomics into slot rows) vs a plain store epilogue, and the standalone finalize kernel alone.
Device time per call (graph replay of 20 calls)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from faster_distributed_training_amd.ops import _native  # noqa: E402
from faster_distributed_training_amd.ops import conv_igemm as ci  # noqa: E402
from roofline_layers import timeit  # noqa: E402


def conv_direct(x, wf, shp, epi, part, tile, kg=1):
    nat = _native.native()
    N, H, W, C = x.shape
    Ho, Wo = ci.out_hw(H, W, shp)
    y = torch.empty(N, Ho, Wo, shp.cout, device=x.device, dtype=torch.bfloat16)
    dh, dw, wt = ci.taps_fwd(shp.k, shp.pad)
    bm, bn, bk = tile
    nat.conv_igemm(x.data_ptr(), 0, 0, 0, 0, wf.data_ptr(), y.data_ptr(), part.data_ptr() if part is not None else 0,
                   part.shape[0] if part is not None else 0, 0, 0, 0, 0, 0, 0, N, H, W, C, Ho, Wo, shp.stride, list(dh),
                   list(dw), list(wt), shp.cout, shp.ntaps * shp.cxp, Ho, Wo, 1, 0, 0, 0, 0, 1.0, epi, 0, 1.0, bm, bn,
                   bk, 1, 0, 0, kg, _native.stream_ptr(), [], [], [])
    return y


def main():
    dev = torch.device("cuda")
    nat = _native.native()
    for (N, H, cin, cout, k, tile) in ((128, 8, 8, 256, 3, (64, 128, 64)), (128, 8, 256, 256, 3, (64, 128, 64)),
                                       (128, 8, 1024, 256, 1, (64, 128, 64)), (128, 4, 512, 2048, 1, (64, 128, 64)),
                                       (128, 32, 64, 256, 1, (128, 128, 32)), (1024, 8, 256, 256, 3, (128, 128, 64))):
        shp = ci.ConvShape(cin, cout, k, 1, k // 2)
        x = torch.randn(N, H, H, shp.cxp, device=dev).to(torch.bfloat16)
        w = torch.randn(cout, cin, k, k, device=dev) / (cin * k * k) ** 0.5
        wf, _ = ci.alloc_packed(shp, dev, dgrad=False)
        ci.pack_weights([(w, wf, None, shp)])
        rows = ci.slot_rows(N * H * H)
        part = torch.zeros(rows, 2, cout, device=dev)
        t_stats = timeit(lambda: conv_direct(x, wf, shp, ci.EPI_STATS, part, tile), 20) * 1e3
        t_store = timeit(lambda: conv_direct(x, wf, shp, ci.EPI_STORE, None, tile), 20) * 1e3
        nat.set_conv_debug_flags(1)
        t_noatom = timeit(lambda: conv_direct(x, wf, shp, ci.EPI_STATS, part, tile), 20) * 1e3
        nat.set_conv_debug_flags(0)
        part64 = torch.zeros(64, 2, cout, device=dev)
        t_256 = None
        if rows == 64:
            # (more slot rows = fewer adders per address; the deterministic-mode path sizes them
            # one per row block: the kernel's slot mask comes from the row count)
            prt = torch.zeros(1 << max(6, (-(-N * H * H // tile[0]) - 1).bit_length()), 2, cout, device=dev)
            _native.native().set_deterministic_mode(True)
            t_256 = timeit(lambda: conv_direct(x, wf, shp, ci.EPI_STATS, prt, tile), 20) * 1e3
            _native.native().set_deterministic_mode(False)
        s, t, sm, sa = (torch.empty(cout, device=dev) for _ in range(4))
        t_fin = timeit(lambda: nat.stats_finalize(part.data_ptr(), rows, cout, float(N * H * H), 0, 1e-3, 0.1, 0, 0, 0,
                                                  0, 0, s.data_ptr(), t.data_ptr(), sm.data_ptr(), sa.data_ptr(), 1,
                                                  _native.stream_ptr()), 20) * 1e3
        print(f"N {N} {H}x{H} {cin}->{cout} k{k} tile {tile} ({rows} slot rows): stats epilogue {t_stats:6.1f} us, "
              f"stats without the atomics {t_noatom:6.1f} us, one slot row per workgroup {t_256 or 0:6.1f} us, "
              f"store epilogue {t_store:6.1f} us, finalize alone {t_fin:5.1f} us", flush=True)
    e = torch.empty(1, device=dev)
    print(f"empty fill kernel: {timeit(lambda: e.fill_(1.0), 20) * 1e3:5.1f} us per launch")


if __name__ == "__main__":
    main()
