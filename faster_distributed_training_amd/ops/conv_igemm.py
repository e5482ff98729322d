"""Host side of the hand-written implicit-GEMM convolution kernels (csrc/kernels/conv_igemm.hip,
csrc/kernels/conv_wgrad.hip).

Tensors are NHWC bf16 (``[N, H, W, C]`` contiguous).  Weights are packed once per step
by ``pack_weights`` from the fp32 OIHW master copy (flat parameter buffer) into

* ``wf``: ``[Cout][KH*KW][Cxp]`` — forward operand, K-contiguous per output channel
  (``Cxp`` = input channels padded to a power of two >= 8, e.g. 3 -> 8 for the stem);
* ``wd``: ``[Cin][KH*KW][Cout]`` — data-gradient operand.

Geometry helpers turn (kernel, stride, pad) into the tap tables the kernels consume:
forward ``ih = oh*S + dh``; dgrad of a stride-1 conv is a conv of the gradient with the
taps mirrored; dgrad of a stride-2 conv is split into 4 output-parity classes.
"""
from __future__ import annotations

import json
import os
from dataclasses import dataclass
from functools import lru_cache

import torch

from . import _native

PRO_NONE, PRO_AFFINE_ACT, PRO_FOLD, PRO_JOIN = 0, 1, 2, 3
EPI_STATS, EPI_ACTBWD, EPI_STORE, EPI_ADD, EPI_JOINBWD = 0, 1, 2, 3, 4


def _sp():
    return _native.stream_ptr()


def _p(t):
    return 0 if t is None else t.data_ptr()


def pad_channels(c: int) -> int:
    p = 8
    while p < c:
        p *= 2
    return p


@lru_cache(maxsize=None)
def taps_fwd(k: int, pad: int):
    dh, dw, wt = [], [], []
    for kh in range(k):
        for kw in range(k):
            dh.append(kh - pad)
            dw.append(kw - pad)
            wt.append(kh * k + kw)
    return dh, dw, wt


@lru_cache(maxsize=None)
def dgrad_classes(k: int, stride: int, pad: int):
    """[(py, px, dh, dw, wt)]: output-parity classes of the transposed convolution.
    For each class the valid taps satisfy (p + pad - kh) % stride == 0 and read the
    gradient at  ho = a + (p + pad - kh) / stride  (a = class-grid row)."""
    out = []
    for py in range(stride):
        for px in range(stride):
            dh, dw, wt = [], [], []
            for kh in range(k):
                if (py + pad - kh) % stride:
                    continue
                for kw in range(k):
                    if (px + pad - kw) % stride:
                        continue
                    dh.append((py + pad - kh) // stride)
                    dw.append((px + pad - kw) // stride)
                    wt.append(kh * k + kw)
            out.append((py, px, dh, dw, wt))
    return out


def pick_tile(M: int, N: int, cands=((128, 128), (128, 64), (64, 128), (64, 64)), want: int = 512, bk: int = 64):
    """Heuristic (BM, BN, BK) when no tuned entry exists: the largest tile that still
    gives ~2 workgroups per CU."""
    best = None
    for bm, bn in cands:
        if N % bn:
            continue
        nb = -(-M // bm) * (N // bn)
        if nb >= want:
            return bm, bn, bk
        if best is None or nb > best[0]:
            best = (nb, bm, bn)
    return best[1], best[2], bk


_TUNED = None
_TUNED_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "conv_tuned.json")


def tune_key(batch: int, h: int, shp) -> str:
    return f"{batch}:{h}:{shp.cin}:{shp.cout}:{shp.k}:{shp.stride}:{shp.pad}"


# Launch record (tests): when a list, every conv launch appends (kind, tune key, tuned entry
# found, (bm, bn, bk), nsplit, K groups) -- which shipped tile-table choices actually ran.
LAUNCH_LOG = None


def _log(kind, batch, h, shp, ent, tile3, ns, kg=1):
    if LAUNCH_LOG is not None:
        LAUNCH_LOG.append((kind, tune_key(batch, h, shp), bool(ent and "tile" in ent), tuple(tile3), int(ns), int(kg)))


def tuned(op: str, batch: int, h: int, shp):
    """Tuned launch config (scripts/tune_conv.py) for this exact problem, or None."""
    global _TUNED
    if _TUNED is None:
        try:
            with open(_TUNED_PATH) as f:
                _TUNED = json.load(f)
        except (OSError, ValueError):
            _TUNED = {}
    ent = _TUNED.get(tune_key(batch, h, shp), {}).get(op)
    return ent


# ---------------------------------------------------------------- split-K
SPLITK = os.environ.get("FDT_SPLITK", "1") != "0"
_SPLITK_WS: dict = {}


def splitk_heuristic(tiles: int, nkt: int, want: int = 512, min_kt: int = 4, cap: int = 8) -> int:
    """Workgroups per output tile for small-M convolutions: enough to put ~2 workgroups on
    each of the 256 CUs, each split still reducing >= min_kt K tiles."""
    if not SPLITK or tiles >= want * 3 // 4:
        return 1
    ns = -(-want // max(tiles, 1))
    return max(1, min(ns, nkt // min_kt, cap))


def splitk_workspace(dev, slab_floats: int, tiles: int):
    """Persistent (slab, tickets) for split-K launches on ``dev``; tickets are zero between
    launches (each tile's last arriver resets its ticket)."""
    ws = _SPLITK_WS.get(dev)
    if ws is None or ws[0].numel() < slab_floats or ws[1].numel() < tiles:
        slab = torch.empty(max(slab_floats, ws[0].numel() if ws else 0), device=dev, dtype=torch.float32)
        cnt = torch.zeros(max(tiles, ws[1].numel() if ws else 0, 4096), device=dev, dtype=torch.int32)
        ws = _SPLITK_WS[dev] = (slab, cnt)
    return ws


def _splitk_args(ent, M, N, K, bm, bn, bk, dev):
    """(nsplit, slab ptr, ticket ptr) for one launch: tuned entry's nsplit, else heuristic."""
    tiles = -(-M // bm) * (N // bn)
    nkt = -(-K // bk)
    ns = int(ent.get("nsplit", 0)) if ent else 0
    if ns <= 0:
        ns = splitk_heuristic(tiles, nkt)
    ns = max(1, min(ns, nkt))
    if ns == 1:
        return 1, 0, 0
    slab, cnt = splitk_workspace(dev, tiles * ns * (bm // 64) * (bn // 64) * 16 * 256, tiles)
    return ns, slab.data_ptr(), cnt.data_ptr()


def _tile3(tile, M, N):
    if tile is None:
        return pick_tile(M, N)
    if len(tile) == 2:
        return tile[0], tile[1], 64
    return tuple(tile[:3])


# register-staged K tiles in flight in the weight-gradient kernel (csrc/kernels/conv_wgrad.hip):
# 4 is instantiated for the small BK = 32 tiles of the small-batch layers; a tuned entry's
# "stages" overrides this default
WG_STAGES = int(os.environ.get("FDT_WG_STAGES", "2"))
# few-split slab-reduced weight gradients (3x3, padded stem) combine their splits in-kernel
# (last arriver per tile) instead of a separate wgrad_reduce launch
WG_FUSED_REDUCE = os.environ.get("FDT_WG_FUSED_REDUCE", "0") == "1"
WG_FUSED_MAX_SPLITS = 8

# K groups (csrc/kernels/conv_igemm_impl.h): 8-wave workgroups whose two 4-wave halves take
# alternate K tiles -- for the small-M layers whose ~256-workgroup grids leave one wave per SIMD
KGROUPS = os.environ.get("FDT_KGROUPS", "1") != "0"
KG_TILES = {(128, 128, 64), (128, 64, 64), (64, 128, 64), (64, 64, 64), (64, 64, 128)}


# prologue-free launches (3x3 convs on materialised operands, plain dgrads) can stage their tiles
# by LDS-DMA into a 3-buffer ring (kg = 3, csrc/kernels/conv_igemm_impl.h): bitwise equal to the
# register-staged path, measured neutral at batch 128 (5.519 vs 5.518 ms) and slower at batch
# 1024 (26.04 -> 26.73 ms; the 32x32 / strided dgrads lose 13-32 %), profiles/r4/ab_glds_* --
# so opt-in
GLDS = os.environ.get("FDT_CONV_GLDS", "0") == "1"


# K-loop form of the implicit-GEMM kernels (conv_igemm_impl.h main loop) for single-group launches:
# "rot" = the rotated loop with a true 2-deep register prefetch (kg 4), "old" = the legacy loop
# (hipcc drains the prefetch at every trip); per layer from the tuned entry's "loop", else this
# default (the legacy form: measured faster for most of the memory-bound batch-1024 layers)
LOOP = os.environ.get("FDT_CONV_LOOP", "old")

# Halo-staged 3x3 stride-1 main loop (csrc/kernels/conv_h3.hip, kg 5): the forward 3x3 convs on
# their materialised inputs and the stride-1 3x3 data gradients on the pre-folded gradient, at
# 256-pixel tiles.  FDT_CONV_H3=0 keeps the implicit-GEMM kernel's tuned tiles;
# FDT_CONV_H3_MIN_TILES: below this many output tiles (small per-GPU batches) the tuned
# implicit-GEMM launch (split-K / K groups) keeps the layer.
H3 = os.environ.get("FDT_CONV_H3", "1") == "1"
H3_MIN_TILES = int(os.environ.get("FDT_CONV_H3_MIN_TILES", "256"))
H3_TILES = {(256, 128), (256, 64), (128, 128)}
# staging of the halo loop: "dma" = LDS-DMA issued a chunk ahead into a second stage (kg 6, 128
# output channels per workgroup: one workgroup per CU), "dma64" = the same at 64 output channels
# per workgroup (78 KB of LDS: TWO workgroups per CU, each double-buffered), "dma1" = LDS-DMA
# into one stage, two workgroups per CU (kg 7; the probe shows the two phase-locked: they load
# and compute together, profiles/r6/h3_probe_1024.txt), "reg" = register-staged (kg 5);
# "auto" = the measured per-shape choice (h3_auto)
H3_LOOP = os.environ.get("FDT_CONV_H3_LOOP", "auto")
H3_KGS = (5, 6, 7, 8)
# the 2- and 4-tap output-parity classes of the stride-2 3x3 data gradients through the halo loop
# (kg 6; H, W = the output-gradient grid); the 1-tap class stays a plain GEMM.  Measured SLOWER
# (scripts/bench_s2.py, profiles/r6/bench_s2_*.txt: batch 1024 32x32 265 -> 318 us, 16x16 197 ->
# 211, 8x8 137 -> 142; whole step 24.53-24.60 -> 24.59-24.73 ms): with 2-4 taps per chunk the halo
# staging is not amortised.  Opt-in (tests keep it correct).
H3_S2 = os.environ.get("FDT_CONV_H3_S2", "0") == "1"


def _h3_kg(kg, W=8):
    if kg in H3_KGS:
        return kg
    return {"dma": 6, "dma64": 6, "auto": 6, "dma1": 7}.get(H3_LOOP, 5)


def h3_tile(N, H, W, shp: "ConvShape", pro, cout, force=False, cx=None, bn=None, s2cls=False):
    """(BM, BN) of the halo 3x3 loop for this launch, or None (csrc/kernels/conv_h3.hip
    h3_supported: 3x3 pad-1 stride-1, prologue-free, whole image rows per 256-pixel tile).
    ``force`` (an explicit kg 5): ignore FDT_CONV_H3 and the small-grid cut-off.  ``cx``: the
    operand's channels (forward: cxp; data gradient: cout), a multiple of 16."""
    if cx is None:
        cx = shp.cxp
    conv_ok = shp.k == 3 and shp.pad == 1 and shp.stride == (2 if s2cls else 1)
    if not (H3 or force) or pro != PRO_NONE or cx % 16 or not conv_ok or W < 4 or W & (W - 1):
        return None
    bm = 256
    M = N * H * W
    if M % bm or bm % W:
        return None
    rb = min(H, bm // W)
    if (rb < H and H % rb) or (rb == H and bm % (H * W)):
        return None
    # halo blocks and the 16-pixel lane-group sets (conv_h3.hip H3Geom / h3_supported)
    nbk, gw = bm // (rb * W), min(W, 16)
    ni = 16 // gw
    bhr = (rb + 2) * (W + 2)
    if ni > 1:
        bhr += ((16 // ni) - bhr % 16 + 16) % 16
        if nbk % ni or rb != H:
            return None
    elif W % 16:
        return None
    if nbk * bhr > bm // 16 * 36:
        return None
    if bn is None:
        bn = 64 if H3_LOOP == "dma64" else 128
    bn = bn if cout % bn == 0 else (64 if cout % 64 == 0 else 0)
    if not bn or (not force and (M // bm) * (cout // bn) < H3_MIN_TILES):
        return None
    return bm, bn


def h3_auto(N, H, W, shp: "ConvShape", pro, cout, cx=None):
    """The halo loop's measured per-shape choice (scripts/bench_h3.py, profiles/r6/bench_h3_*.txt):
    ((BM, BN), kg) or None for the implicit-GEMM kernel.  At 32x32 the double-buffered 64-channel
    tiles (two workgroups per CU); at 16x16 / 8x8 the single-stage 128-channel tiles when the grid
    holds >= 512 of them, else (16x16 at the 8-GPU share) the 64-channel double-buffered tiles;
    at 4x4 the double-buffered 128-channel tiles over >= 256 tiles; smaller grids (8x8 / 4x4 at
    batch 128) stay on the tuned implicit-GEMM launches."""
    if H3_LOOP != "auto":
        t = h3_tile(N, H, W, shp, pro, cout, cx=cx)
        return None if t is None else (t, _h3_kg(None, W))
    if h3_tile(N, H, W, shp, pro, cout, force=True, cx=cx, bn=64) is None:
        return None
    tiles128 = (N * H * W // 256) * (cout // 128) if cout % 128 == 0 else 0
    if W >= 32:
        return (256, 64), 6
    if W >= 8:
        if tiles128 >= 512:
            return (256, 128), 7
        return ((256, 64), 6) if W >= 16 else None
    return ((256, 128), 6) if tiles128 >= 256 else None


def _loop_kg(ent, kgv):
    """kg 1 -> 4 when the launch takes the rotated K loop"""
    lp = (ent.get("loop") if ent else None) or LOOP
    return 4 if (kgv == 1 and lp == "rot") else kgv


def _kg(ent, kg, tile3, ns, K, pro=None):
    """K groups of one launch: explicit ``kg``, else the tuned entry's, else 1 (3 = the
    LDS-DMA ring, prologue-free launches only)."""
    if kg is None:
        kg = int(ent.get("kg", 1)) if ent else 1
        if GLDS and pro == PRO_NONE and kg != 2:
            kg = 3
    if kg == 3:
        return 3 if pro == PRO_NONE else 1
    bk = tile3[2]
    if not KGROUPS or kg != 2 or ns != 1 or tuple(tile3) not in KG_TILES or -(-K // bk) < 2:
        return 1
    return 2


@dataclass
class ConvShape:
    cin: int
    cout: int
    k: int
    stride: int
    pad: int

    @property
    def cxp(self):
        return pad_channels(self.cin)

    @property
    def ntaps(self):
        return self.k * self.k


def out_hw(h, w, shp: ConvShape):
    return ((h + 2 * shp.pad - shp.k) // shp.stride + 1, (w + 2 * shp.pad - shp.k) // shp.stride + 1)


STAT_SLOTS = 64  # csrc/kernels/common.h kStatSlots

def _finalize_standalone(nat, kind, part, nq, C, fptr, fval):
    """The statistics consumer launched right after its producer conv: kind 1 = forward
    batch-norm finalize, kind 2 = BN-backward coefficients.  (Folding it into the conv as a
    last-arriver epilogue was measured slower: README, performance notes.)"""
    if kind == 1:  # fptr: gamma beta rm rv nbt s t sm sa ; fval: mode eps momentum count
        nat.stats_finalize(part.data_ptr(), part.shape[0], C, float(fval[3]), int(fval[0]), float(fval[1]),
                           float(fval[2]), *fptr[:9], 1, _sp())
    else:  # per unit: fptr sm sa gamma alpha beta gg gb ; fval mode eps count
        a = [int(fval[0]), float(fval[1]), float(fval[2]), *fptr[0:7]]
        b = [int(fval[3]), float(fval[4]), float(fval[5]), *fptr[7:14]]
        nat.stats_bwd_finalize(part.data_ptr(), part.shape[0], nq, C, *a, *b, _sp())


# large-M 3x3 convolutions (forward stats epilogue, BN-backward dgrad epilogue) spread their
# workgroups over this many slot rows: at batch 1024 the 64-row layout's atomic contention costs
# the 32x32 / 16x16 3x3 convs 4-10 us each in isolation, more than the longer finalize
# (scripts/conv_probe3.py, profiles/r5/probe3_*.txt) -- but the whole step measured 25.37 ->
# 25.44 ms (256 rows) / 25.56 (1024), profiles/r5/wide_rows_*.json: off by default (0)
WIDE_ROWS = int(os.environ.get("FDT_STAT_WIDE_ROWS", "0"))
WIDE_MIN_M = 1 << 18


def slot_rows(M: int | None = None, wide: bool = False) -> int:
    """Statistics slot rows for a producer over M output rows: rows shared by workgroups
    (block index mod rows) -- STAT_SLOTS, or fewer for small M (a conv has at most M/64 row
    blocks, and fewer rows are less for the finalize to read), or WIDE_ROWS for a ``wide``
    (3x3) producer over >= WIDE_MIN_M rows -- or in deterministic mode one row per workgroup
    (the BN-backward kernels cap their grid to the rows)."""
    if not _native.deterministic():
        if M is None:
            return STAT_SLOTS
        if wide and WIDE_ROWS > STAT_SLOTS and M >= WIDE_MIN_M:
            return WIDE_ROWS
        need = min(STAT_SLOTS, max(1, -(-int(M) // 64)))
        return 1 << (need - 1).bit_length()
    assert M is not None, "deterministic mode sizes the slots by the producer's row count"
    need = max(STAT_SLOTS, -(-int(M) // 64))
    return 1 << (need - 1).bit_length()


def stat_slots(nq: int, C: int, device, M: int | None = None, wide: bool = False) -> torch.Tensor:
    """A fresh zeroed statistics-slot buffer [slot_rows(M, wide), nq, C] (the engine instead
    reuses one persistent workspace that its finalize kernels re-zero)."""
    return torch.zeros(slot_rows(M, wide), nq, C, device=device, dtype=torch.float32)


_NOLAZY = ([], [])


def conv_fwd(x, wf, shp: ConvShape, s=None, t=None, act=0, alpha=1.0, tile=None, part=None, nsplit=None,
             fin=None, kg=None, lazy=None):
    """y = conv(act(x*s+t)) (or conv(x) when s is None and act == 0); returns
    (y [N,Ho,Wo,Cout] bf16, part [STAT_SLOTS,2,Cout] fp32 slots whose row sum is
    (sum y, sum y^2)).  ``part``: a zeroed slot buffer to accumulate into.
    ``fin`` = (fptr, fval): then finalise the batch-norm statistics (stats_finalize
    arguments: gamma beta run_mean run_var nbt s t save_mean save_aux / mode eps momentum
    count) and re-zero the slots.
    ``lazy`` = (ptr list, value list) of the INPUT's statistics left in its producer's slot rows
    (bn_math.h LazyStats): the prologue finalises them itself (s / t unused, written by
    workgroup 0 for the backward)."""
    nat = _native.native()
    N, H, W, C = x.shape
    assert C == shp.cxp and x.dtype == torch.bfloat16 and x.is_contiguous()
    Ho, Wo = out_hw(H, W, shp)
    M = N * Ho * Wo
    pro = PRO_AFFINE_ACT if (s is not None or act != 0 or lazy is not None) else PRO_NONE
    ent = None
    h3 = None
    if kg in H3_KGS:
        t3 = h3_tile(N, H, W, shp, pro, shp.cout, True)
        h3 = None if t3 is None else (t3, kg)
    elif kg is None and tile is None and H3:
        h3 = h3_auto(N, H, W, shp, pro, shp.cout)
    if tile is None and h3 is None:
        ent = tuned(f"fwd{pro}", N, H, shp) or tuned("fwd", N, H, shp)
        tile = tuple(ent["tile"]) if ent else None
    if h3 is not None:
        ent, ((bm, bn), kgv), bk = {"loop": "old"}, h3, 16
        ns, slab_p, cnt_p = 1, 0, 0
    else:
        bm, bn, bk = _tile3(tile, M, shp.cout)
        if nsplit is not None:
            ent = {"nsplit": nsplit}
        ns, slab_p, cnt_p = _splitk_args(ent, M, shp.cout, shp.ntaps * C, bm, bn, bk, x.device)
        kgv = _kg(ent, kg, (bm, bn, bk), ns, shp.ntaps * C, pro)
    _log("fwd", N, H, shp, ent, (bm, bn, bk), ns, kgv)
    y = torch.empty(N, Ho, Wo, shp.cout, device=x.device, dtype=torch.bfloat16)
    if part is None:
        part = stat_slots(2, shp.cout, x.device, M)
    dh, dw, wt = taps_fwd(shp.k, shp.pad)
    if pro == PRO_AFFINE_ACT and s is None and lazy is None:
        s = torch.ones(C, device=x.device, dtype=torch.float32)
        t = torch.zeros(C, device=x.device, dtype=torch.float32)
    lz = lazy if lazy is not None else _NOLAZY
    nat.conv_igemm(x.data_ptr(), 0, _p(s), _p(t), 0, wf.data_ptr(), y.data_ptr(), part.data_ptr(), part.shape[0],
                   0, 0, 0, 0, 0, 0,
                   N, H, W, C, Ho, Wo, shp.stride, list(dh), list(dw), list(wt), shp.cout, shp.ntaps * shp.cxp,
                   Ho, Wo, 1, 0, 0, pro, int(act), float(alpha), EPI_STATS, 0, 1.0, bm, bn, bk, ns, slab_p, cnt_p,
                   _loop_kg(ent, kgv), _sp(), lz[0], lz[1], [])
    if fin is not None:
        _finalize_standalone(nat, 1, part, 2, shp.cout, fin[0], fin[1])
    return y, part


def conv_fwd_join(y, r, s, t, s2, t2, wf, shp: ConvShape, jout, jmask=None, tile=None, part=None, nsplit=None,
                  fin=None, kg=None, lazy=None, lazy2=None):
    """1x1 stride-1 forward conv of a residual block's joined output, computed on the fly:
    the operand is a = relu(y*s + t + (r*s2 + t2 if s2 is not None else r)) -- the previous
    block's join (BN'd residual branch y + BN'd or identity shortcut r).  ``jout`` receives
    ``a`` (bf16, the block output the next join and the backward read) and ``jmask`` its
    ReLU bit mask (None: not stored), written once by the first output-channel tile; the
    standalone join kernel and this conv's re-read of ``a`` become one pass.  Returns
    (conv output, statistics slots) like ``conv_fwd``.  ``lazy`` / ``lazy2``: the branches'
    statistics left in their producers' slot rows (see ``conv_fwd``; s / t and s2 / t2 unused)."""
    nat = _native.native()
    N, H, W, C = y.shape
    assert shp.k == 1 and shp.stride == 1 and shp.pad == 0 and C == shp.cin == shp.cxp
    for tt in (y, r, jout):
        assert tt.dtype == torch.bfloat16 and tt.is_contiguous() and tuple(tt.shape) == (N, H, W, C)
    assert (s2 is None) == (t2 is None) and (lazy2 is None or lazy is not None)
    assert jmask is None or (jmask.dtype == torch.uint8 and jmask.numel() * 8 >= y.numel())
    M = N * H * W
    ent = None
    if tile is None:
        ent = tuned("fwd3", N, H, shp) or tuned("fwd0", N, H, shp) or tuned("fwd", N, H, shp)
        tile = tuple(ent["tile"]) if ent else None
    bm, bn, bk = _tile3(tile, M, shp.cout)
    if nsplit is not None:
        ent = {"nsplit": nsplit}
    ns, slab_p, cnt_p = _splitk_args(ent, M, shp.cout, C, bm, bn, bk, y.device)
    kgv = _kg(ent, kg, (bm, bn, bk), ns, C)
    _log("fwd_join", N, H, shp, ent, (bm, bn, bk), ns, kgv)
    out = torch.empty(N, H, W, shp.cout, device=y.device, dtype=torch.bfloat16)
    if part is None:
        part = stat_slots(2, shp.cout, y.device, M)
    l1 = lazy if lazy is not None else _NOLAZY
    l2 = lazy2 if lazy2 is not None else _NOLAZY
    nat.conv_igemm_join(y.data_ptr(), r.data_ptr(), _p(s), _p(t), _p(s2), _p(t2), wf.data_ptr(),
                        out.data_ptr(), part.data_ptr(), part.shape[0], jout.data_ptr(), _p(jmask), N, H, W, C,
                        shp.cout, shp.ntaps * shp.cxp, bm, bn, bk, ns, slab_p, cnt_p, _loop_kg(ent, kgv), _sp(),
                        l1[0], l1[1], l2[0], l2[1])
    if fin is not None:
        _finalize_standalone(nat, 1, part, 2, shp.cout, fin[0], fin[1])
    return out, part


def conv_dgrad(g, y, al, be, wd, shp: ConvShape, x_shape, epi=EPI_STORE, out=None, ex=None, es=None, et=None,
               act=0, alpha=1.0, tile=None, part=None, nsplit=None, gs=None, jmask=None, jyb=None, jout=None,
               coef=None, kg=None, jz=None):
    """Data gradient of y = conv(a): dA = conv^T(g*gs + al + be*y)  (gs None: 1).

    epi: EPI_STORE -> write dA; EPI_ADD -> out += dA; EPI_ACTBWD -> through the lazy
    input a = act(ex*es + et): out = dA*act'(.)*es, returns statistics slots
    [STAT_SLOTS, 2, Cin] whose row sum is (sum g_pre*ex, sum g_pre) (``part``: a zeroed
    slot buffer to accumulate into; every parity class of a strided conv adds to it);
    EPI_JOINBWD -> out (the gradient of a residual block's output, this dgrad completes it)
    becomes g_pre = (out + dA) * act'(join) with act' from ``jmask`` (ReLU bit mask) or
    ``jout`` (the join output, CELU), and ``part`` [STAT_SLOTS, 3, Cin] receives
    (sum g_pre*ex, sum g_pre, sum g_pre*jyb) -- ex / jyb = the block's residual / shortcut
    branch outputs (jyb None: identity shortcut).  CELU joins take act' from the recomputed fp32
    pre-activation instead of ``jout`` (z mode): ``es`` / ``et`` = the residual branch's BN (s, t)
    and ``jz`` = (sb, tb, xid) -- the shortcut's BN (s, t) or, identity shortcut, (None, None,
    the block input).
    ``coef`` = (fptr, fval) with EPI_ACTBWD / EPI_JOINBWD: then turn the statistics into the
    producer units' BN-backward coefficients (stats_bwd_finalize arguments, units A and B:
    save_mean save_aux gamma alpha beta ggamma gbeta / mode eps count)."""
    nat = _native.native()
    N, Hy, Wy, Cy = g.shape
    assert Cy == shp.cout and g.is_contiguous() and (y is None or y.is_contiguous())
    Nx, Hx, Wx, Cx = x_shape
    assert Cx == shp.cin
    if out is None:
        out = torch.empty(N, Hx, Wx, shp.cin, device=g.device, dtype=torch.bfloat16)
    if epi == EPI_ACTBWD and part is None:
        part = stat_slots(2, shp.cin, g.device, Nx * Hx * Wx)
    if epi == EPI_JOINBWD:
        assert shp.stride == 1 and ex is not None and part is not None and (
            jmask is not None or jout is not None or jz is not None)
        assert (jz is None) == (es is None), "z mode: es / et with jz"
        if jz is not None:
            assert act == 2 and et is not None and len(jz) == 3
            assert (jz[0] is not None and jz[1] is not None) if jyb is not None else jz[2] is not None
            if jz[2] is not None:
                assert jz[2].dtype == torch.bfloat16 and jz[2].is_contiguous() and tuple(jz[2].shape) == tuple(x_shape)
    ent = None
    h3ok = kg in H3_KGS or (kg is None and tile is None)
    if tile is None:
        pro = PRO_FOLD if al is not None else PRO_NONE
        e = EPI_STORE if epi in (EPI_ADD, EPI_JOINBWD) else epi
        ent = tuned(f"dgrad{pro}{e}", N, Hx, shp) or tuned("dgrad", N, Hx, shp)
        tile = tuple(ent["tile"]) if ent else None
    if nsplit is not None:
        ent = {"nsplit": nsplit}
    classes = dgrad_classes(shp.k, shp.stride, shp.pad)
    assert coef is None or epi in (EPI_ACTBWD, EPI_JOINBWD)
    for (py, px, dh, dw, wt) in classes:
        Ha = (Hx - py + shp.stride - 1) // shp.stride
        Wa = (Wx - px + shp.stride - 1) // shp.stride
        M = N * Ha * Wa
        if len(dh) == 0 and epi == EPI_ADD:
            continue
        pro = PRO_FOLD if al is not None else PRO_NONE  # al None: g is already folded
        h3 = None
        if h3ok and epi in (EPI_ACTBWD, EPI_STORE) and len(dh) == 9:
            if kg in H3_KGS:
                t3 = h3_tile(N, Hx, Wx, shp, pro, shp.cin, True, cx=Cy)
                h3 = None if t3 is None else (t3, kg)
            elif H3:
                h3 = h3_auto(N, Hx, Wx, shp, pro, shp.cin, cx=Cy)
        elif (h3ok and epi in (EPI_ACTBWD, EPI_STORE) and len(dh) in (2, 4) and shp.k == 3 and shp.stride == 2
              and Ha == Hy and Wa == Wy and (H3_S2 or kg in H3_KGS)):
            t3 = h3_tile(N, Ha, Wa, shp, pro, shp.cin, force=kg in H3_KGS, cx=Cy, s2cls=True)
            h3 = None if t3 is None else (t3, 6)
        if h3 is not None:
            ((bm, bn), kgv), bk = h3, 16
            ns, slab_p, cnt_p = 1, 0, 0
        else:
            bm, bn, bk = _tile3(tile, M, shp.cin)
            ns, slab_p, cnt_p = _splitk_args(ent, M, shp.cin, len(dh) * Cy, bm, bn, bk, g.device)
            kgv = _kg(ent, kg, (bm, bn, bk), ns, len(dh) * Cy, pro)
        _log("dgrad", N, Hx, shp, ent, (bm, bn, bk), ns, kgv)
        assert gs is None or pro == PRO_FOLD, "gs needs the fold prologue (al/be)"
        nat.conv_igemm(g.data_ptr(), _p(y) if pro == PRO_FOLD else 0, _p(al), _p(be), _p(gs), wd.data_ptr(),
                       out.data_ptr(), _p(part) if epi in (EPI_ACTBWD, EPI_JOINBWD) else 0,
                       part.shape[0] if part is not None else 0, _p(ex), _p(es), _p(et),
                       _p(jmask), _p(jyb), _p(jout), N, Hy, Wy, Cy, Ha, Wa, 1,
                       list(dh), list(dw), list(wt), shp.cin, shp.ntaps * shp.cout, Hx, Wx, shp.stride, py, px,
                       pro, 0, 1.0, epi, int(act), float(alpha), bm, bn, bk, ns, slab_p, cnt_p, _loop_kg(ent, kgv),
                       _sp(), [], [], [_p(v) for v in jz] if jz is not None else [])
    if coef is not None:
        _finalize_standalone(nat, 2, part, 3 if epi == EPI_JOINBWD else 2, shp.cin, coef[0], coef[1])
    return out, (part if epi in (EPI_ACTBWD, EPI_JOINBWD) else None)


# Halo-staged 3x3 stride-1 weight gradient (csrc/kernels/conv_wh3.hip) on the materialised
# operands (folded gradient, normalised input): a workgroup owns (co, ci) x all nine taps and
# stages each 128-pixel chunk's input halo once instead of once per tap.  FDT_WGRAD_H3=0 keeps
# the implicit-GEMM weight gradient; FDT_WGRAD_H3_WGS: target workgroups (one per CU: ~110 KB
# of LDS each), the pixel split follows.
WH3 = os.environ.get("FDT_WGRAD_H3", "1") == "1"
WH3_WGS = int(os.environ.get("FDT_WGRAD_H3_WGS", "256"))
# ... and at least this many 128-pixel chunks per workgroup (fewer splits: a smaller fp32 slab to
# write and reduce when the pixel count is small)
WH3_MIN_CPS = int(os.environ.get("FDT_WGRAD_H3_MIN_CPS", "1"))
WH3_PX = 128
# register-pipelined fragments (conv_wh3.hip PIPE) and waves per (co, ci) block (TS: 2 = eight
# waves, each with half the tap accumulators; not combinable with PIPE).  Both measured neutral
# or slower at the final register allocation (profiles/r6/wh3_ts*_p*_*.txt): off by default
WH3_PIPE = os.environ.get("FDT_WGRAD_H3_PIPE", "0") == "1"
WH3_TS = int(os.environ.get("FDT_WGRAD_H3_TS", "1"))


def wh3_plan(N, H, W, shp: "ConvShape", cx, fold=False, xaff=False, force=False):
    """((BMC, BNC), nsplit) of the halo weight gradient, or None (conv_wh3.hip's geometry:
    3x3 pad-1 stride-1, power-of-two images >= 4x4, 128-pixel chunks of whole rows whose halo fits
    288 rows, no fused fold / input transform)."""
    if not (WH3 or force) or fold or xaff or shp.k != 3 or shp.stride != 1 or shp.pad != 1:
        return None
    if H < 4 or W < 4 or H & (H - 1) or W & (W - 1) or W > WH3_PX:
        return None
    M = N * H * W
    if M % WH3_PX:
        return None
    rb = min(H, WH3_PX // W)
    if (WH3_PX // (rb * W)) * (rb + 2) * (W + 2) > WH3_PX // 16 * 36:
        return None
    co = shp.cout
    if co % 128 == 0 and cx % 32 == 0:
        t = (128, 32)
    elif co % 64 == 0 and cx % 64 == 0:
        t = (64, 64)
    else:
        return None
    # measured (scripts/bench_h3.py --only wgrad, profiles/r6/bench_wh3_*.txt): a win on every
    # batch-1024 layer (32x32 211 -> 118 us, 16x16 156 -> 95, 8x8 114 -> 94, 4x4 119 -> 94) and on
    # the 32x32 / 16x16 layers at batch 128; the small 8x8 / 4x4 layers at batch 128 (~30 us,
    # latency-bound either way) keep the implicit-GEMM kernel
    if not force and W < 16 and M * co * cx < (1 << 31):
        return None
    tiles = (co // t[0]) * (cx // t[1])
    chunks = M // WH3_PX
    ns = max(1, min(chunks // max(1, WH3_MIN_CPS), WH3_WGS // tiles))
    cps = -(-chunks // ns)
    return t, -(-chunks // cps)


def wgrad_split(M: int, tiles: int, want: int = 512, min_px: int = 1024) -> int:
    s = max(1, want // max(tiles, 1))
    s = min(s, max(1, M // min_px))
    return s


def conv_wgrad(g, y, al, be, x, shp: ConvShape, out, xs=None, xt=None, act=0, alpha=1.0, accumulate=False,
               tile=None, nsplit=None, slab=None, gs=None, h3=None):
    """out (fp32 OIHW [Cout, Cin, k, k]) = dL/dW of y = conv(act(x*xs+xt)) given
    g (gradient wrt y, corrected to g*gs + al + be*y in the kernel; gs None: 1).  ``h3``: the
    halo weight gradient (``wh3_plan``) -- None = where it applies (no explicit tile), True =
    forced, False = the implicit-GEMM kernel."""
    nat = _native.native()
    N, Hy, Wy, Cy = g.shape
    Nx, H, W, Cx = x.shape
    assert Cx == shp.cxp and Cy == shp.cout
    M = N * Hy * Wy
    ldw = shp.ntaps * shp.cxp
    wp = None
    if h3 is True or (h3 is None and tile is None and nsplit is None):
        wp = wh3_plan(N, H, W, shp, Cx, al is not None, xs is not None or act != 0, force=h3 is True)
        assert wp is not None or h3 is not True, "halo weight gradient: unsupported geometry"
    if wp is not None:
        assert g.is_contiguous() and x.is_contiguous() and g.dtype == torch.bfloat16 and x.dtype == torch.bfloat16
        assert out.is_contiguous() and tuple(out.shape) == (shp.cout, shp.cin, 3, 3)
        (bmc, bnc), ns = wp
        _log("wgrad_h3", N, H, shp, None, (bmc, bnc, WH3_PX), ns, 9)  # (kg 9 marks the halo wgrad)
        if slab is None or slab.numel() < ns * shp.cout * ldw:
            slab = torch.empty(ns * shp.cout * ldw, device=g.device, dtype=torch.float32)
        nat.conv_wgrad_h3(g.data_ptr(), x.data_ptr(), slab.data_ptr(), N, H, W, Cx, shp.cout, bmc, bnc, ns,
                          int(WH3_PIPE) | (4 if WH3_TS == 2 else 0), _sp())
        nat.wgrad_reduce(slab.data_ptr(), out.data_ptr(), ns, shp.cout, shp.cin, shp.ntaps, shp.cxp,
                         int(accumulate), _sp())
        return out
    ent = None
    if tile is None:
        ent = tuned(f"wgrad{int(al is not None)}{int(xs is not None or act != 0)}", N, H, shp) or \
            tuned("wgrad", N, H, shp)
        if ent:
            tile = tuple(ent["tile"])
            nsplit = nsplit or ent["nsplit"]
    if tile is None:
        bm = 128 if shp.cout % 128 == 0 else 64
        bn = 128 if ldw >= 128 else 64
        bk = 64
    elif len(tile) == 2:
        (bm, bn), bk = tile, 64
    else:
        bm, bn, bk = tile
    tiles = (shp.cout // bm) * (-(-ldw // bn))
    ns = nsplit or wgrad_split(M, tiles)
    _log("wgrad", N, H, shp, ent, (bm, bn, bk), ns)
    # 1x1 without channel padding: the slab row layout IS OIHW -> every split adds into
    # `out` with fp32 atomics (no slab, no reduce launch); deterministic mode keeps the
    # ordered slab reduction
    direct = shp.ntaps == 1 and shp.cxp == shp.cin and out.is_contiguous() and not _native.deterministic()
    if direct:
        if not accumulate:
            out.zero_()
        slab = out
    fused = (WG_FUSED_REDUCE and not direct and 1 < ns <= WG_FUSED_MAX_SPLITS and out.is_contiguous())
    if fused:
        # splits combined in-kernel by the last arriver of each tile (no wgrad_reduce launch):
        # partial tiles in register order in the persistent split-K workspace
        tiles = (shp.cout // bm) * (-(-ldw // bn))
        slab, cnt = splitk_workspace(g.device, tiles * ns * bm * bn, tiles)
    elif not direct and (slab is None or slab.numel() < ns * shp.cout * ldw):
        slab = torch.empty(ns * shp.cout * ldw, device=g.device, dtype=torch.float32)
    dh, dw, _ = taps_fwd(shp.k, shp.pad)
    if xs is None and act != 0:
        xs = torch.ones(Cx, device=x.device, dtype=torch.float32)
        xt = torch.zeros(Cx, device=x.device, dtype=torch.float32)
    assert gs is None or al is not None, "gs needs the fold (al/be)"
    stages = int(ent.get("stages", WG_STAGES)) if ent else WG_STAGES
    nat.conv_wgrad(g.data_ptr(), _p(y), _p(al), _p(be), _p(gs), x.data_ptr(), _p(xs), _p(xt), slab.data_ptr(),
                   N, H, W, Cx, Hy, Wy, shp.stride, list(dh), list(dw), shp.cout, ldw, int(act), float(alpha),
                   bm, bn, bk, ns, int(direct), stages, out.data_ptr() if fused else 0,
                   cnt.data_ptr() if fused else 0, shp.cin, int(accumulate), _sp())
    if not direct and not fused:
        nat.wgrad_reduce(slab.data_ptr(), out.data_ptr(), ns, shp.cout, shp.cin, shp.ntaps, shp.cxp,
                         int(accumulate), _sp())
    return out


def pack_weights(entries):
    """entries: iterable of (w fp32 OIHW, wf bf16 or None, wd bf16 or None, ConvShape); one
    launch (a None layout is skipped)."""
    nat = _native.native()
    src, wf, wd, co, ci, cx, nt = [], [], [], [], [], [], []
    for w, f, d, shp in entries:
        assert w.is_contiguous() and w.dtype == torch.float32
        src.append(w.data_ptr())
        wf.append(_p(f))
        wd.append(_p(d))
        co.append(shp.cout)
        ci.append(shp.cin)
        cx.append(shp.cxp)
        nt.append(shp.ntaps)
    if src:
        nat.pack_weights(src, wf, wd, co, ci, cx, nt, _sp())


def alloc_packed(shp: ConvShape, device, dgrad=True, fwd=True):
    wf = torch.empty(shp.cout, shp.ntaps, shp.cxp, device=device, dtype=torch.bfloat16) if fwd else None
    wd = torch.empty(shp.cin, shp.ntaps, shp.cout, device=device, dtype=torch.bfloat16) if dgrad else None
    return wf, wd
