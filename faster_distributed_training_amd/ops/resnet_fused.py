"""MI355X execution engine for the ResNet family: the whole network body (stem + all residual
blocks) is ONE autograd node whose forward and backward are explicit sequences of the
hand-written HIP kernels.

Why one node: the reference runs ~7 kernels and 3-4 activation passes per FusedConvBN in
forward and ~15 in backward, recomputing the conv (resnet.py:72-113, survey CS4).  Here
each convolution is one implicit-GEMM MFMA kernel whose prologue applies the producer's
batch-norm + activation while staging the operand (a conv output is never normalised in
memory) and whose epilogue emits the per-channel statistics of its own output.  Backward
is likewise one dgrad kernel (prologue: the batch-norm backward correction
g + alpha + beta*y; epilogue: the consumer activation backward + the producer's
statistics reductions) and one wgrad kernel per convolution.  Owning the whole body lets
the engine

* accumulate the two data-gradient contributions of a block input (residual path and
  shortcut) inside the second dgrad's epilogue (no autograd sum kernel),
* write weight / BN-affine gradients straight into the flat gradient buffer and signal
  DDP bucket readiness itself (``grad_ready``), in backward order,
* pack every conv weight to bf16 GEMM layouts in one launch per step,
* stay free of host synchronisation and allocation-order dependence, so a whole train
  step can be captured in a HIP graph.

Numerics follow the reference exactly where it defines the model: FusedConvBN uses batch
statistics in train AND eval with unbiased variance and (y-mean)/(sqrt(var)+1e-3)
(resnet.py:75-100); nn.BatchNorm2d uses biased variance, affine, running statistics with
momentum (resnet.py:204-206, 221-223).  Compute is bf16 MFMA with fp32 accumulation and
fp32/fp64 statistics.
"""
from __future__ import annotations

import os

import torch
import torch.nn as nn

from . import _native
from . import conv_igemm as ci
from ..parallel import graphs as _graphs

ACT_NONE, ACT_RELU, ACT_CELU = 0, 1, 2
# materialise the normalised input / folded gradient of 3x3 convs once (see forward/backward)
MATERIALIZE_3X3 = os.environ.get("FDT_MATERIALIZE_3X3", "1") != "0"
# run a block's ReLU join inside the next block's first 1x1 conv (PRO_JOIN prologue) instead
# of a standalone pass (see ResNetBodyFn.forward)
JOIN_FOLD = os.environ.get("FDT_JOIN_FOLD", "1") != "0"
# widest next-block 1x1 (output channels) that still takes the join fold (_join_fold_tile: one
# output-channel tile, and 256 only at >= 65536 rows)
JOIN_FOLD_MAX = int(os.environ.get("FDT_JOIN_FOLD_MAX", "256"))
# ... and, past 64 output channels without a tuned "fwd3" entry, only over at least this many rows
# (batch 128's stage-2 joins measured 0.2 % slower folded: profiles/r5/joinfold_bs128_*.json)
JOIN_FOLD_MIN_M = int(os.environ.get("FDT_JOIN_FOLD_MIN_M", str(1 << 18)))
# run the classifier head (average pool + fc, bf16 autocast numerics) as two engine kernels
# inside the body's graphs instead of eager PyTorch ops (see csrc/kernels/head.hip)
FUSED_HEAD = os.environ.get("FDT_FUSED_HEAD", "1") != "0"
MODE_FCBN, MODE_BN_TRAIN, MODE_BN_EVAL = 0, 1, 2
BF16 = torch.bfloat16
# Lazy batch statistics (csrc/kernels/bn_math.h LazyStats): a unit whose statistics fit a few
# slot rows leaves them there and its CONSUMER (next conv's prologue, the 3x3 materialisation,
# the residual join) finalises them while staging its input -- no standalone finalize launch
# (and its kernel boundary) between producer and consumer.  Budget: slot rows x channels a
# consumer workgroup reduces (rows = one per 32 producer row blocks, so <= 32 fp32 atomic adders
# per slot address, the full-rate regime of the memory-side atomics).
LAZY_STATS = os.environ.get("FDT_LAZY_STATS", "0") == "1"
LAZY_BUDGET = int(os.environ.get("FDT_LAZY_BUDGET", "2048"))
# which consumers finalise lazily: "elementwise" (the 3x3 materialisation / stem pass and the
# residual join pass) or "all" (also the conv prologues: AFFINE_ACT / JOIN)
LAZY_SCOPE = os.environ.get("FDT_LAZY_SCOPE", "elementwise")

# Parameters whose gradient the engine writes itself call these hooks (the DDP reducer
# registers here in addition to autograd's post-accumulate-grad hooks).  A "deferrable"
# hook (the reducer's) takes ``defer=True`` and returns its GPU action (a bucket
# all-reduce) instead of launching it, so the engine can first join its weight-gradient
# stream (below) -- and, while capturing, cut the HIP graph there.
_GRAD_READY_HOOKS: dict[int, list] = {}


def register_grad_ready_hook(param, fn, deferrable=False):
    ent = (fn, bool(deferrable))
    _GRAD_READY_HOOKS.setdefault(id(param), []).append(ent)

    class _Handle:
        def remove(self_inner):
            lst = _GRAD_READY_HOOKS.get(id(param), [])
            if ent in lst:
                lst.remove(ent)
    return _Handle()


# While a backward is being captured into HIP graphs (parallel/graphs.py recording),
# deferrable hooks return their GPU action; the recorder cuts the graph there so the action
# runs between two graph segments on every replay (communication keeps overlapping backward).
def grad_ready(param):
    hooks = _GRAD_READY_HOOKS.get(id(param), ())
    if not hooks:
        return
    rec = _graphs.active()
    acts = []
    for fn, deferrable in hooks:
        if deferrable:
            a = fn(param, defer=True)
            if a is not None:
                acts.append(a)
        else:
            fn(param)
    if not acts:
        return
    br = _ACTIVE_BRANCH
    if br is not None and torch.cuda.current_stream() == br.main:
        # a bucket completed by a gradient the main stream wrote (BN parameters): its other
        # members may be weight gradients still running on the weight-gradient branch
        br.join(keep=True)
    if rec is not None:
        rec.cut(acts)
    else:
        for a in acts:
            a()


def _sp():
    return _native.stream_ptr()


def _p(t):
    return 0 if t is None else t.data_ptr()


def _f32(n, dev):
    return torch.empty(n, device=dev, dtype=torch.float32)


class Unit:
    """One convolution + its normalisation."""

    def __init__(self, conv, bn, act_out):
        from ..models.resnet import FusedConvBN
        if isinstance(conv, FusedConvBN):
            self.w = conv.conv_weight
            stride, pad = 1, conv.padding
            self.bn = None
            self.eps = conv.eps
        else:
            assert isinstance(conv, nn.Conv2d) and isinstance(bn, nn.BatchNorm2d)
            self.w = conv.weight
            stride, pad = conv.stride[0], conv.padding[0]
            self.bn = bn
            self.eps = bn.eps
        cout, cin, k, _ = self.w.shape
        self.shp = ci.ConvShape(cin, cout, k, stride, pad)
        self.act_out = act_out  # activation the consumer applies to this unit's normalised output
        self.wf = self.wd = None

    def mode(self, training):
        if self.bn is None:
            return MODE_FCBN
        use_batch = training or not self.bn.track_running_stats
        return MODE_BN_TRAIN if use_batch else MODE_BN_EVAL

    def ensure_packed_buffers(self, dev, need_dgrad):
        need_wd = need_dgrad and self.shp.cin >= 8
        if self.wf is None or self.wf.device != dev:
            self.wf, self.wd = ci.alloc_packed(self.shp, dev, dgrad=need_wd)
        elif need_wd and self.wd is None:
            # (an eval / no-grad forward packs no dgrad layout; a later train step needs it)
            self.wd = ci.alloc_packed(self.shp, dev, dgrad=True, fwd=False)[1]


def _act_of(m):
    if isinstance(m, nn.ReLU):
        return (ACT_RELU, 1.0)
    if isinstance(m, nn.CELU):
        return (ACT_CELU, float(m.alpha))
    return None


def _chain(seq: nn.Sequential):
    """nn.Sequential of (FusedConvBN | Conv2d+BatchNorm2d | activation) -> [Unit]."""
    mods = list(seq)
    units = []
    i = 0
    while i < len(mods):
        m = mods[i]
        a = _act_of(m)
        if a is not None:
            assert units, "activation before any conv"
            units[-1].act_out = a
            i += 1
            continue
        if isinstance(m, nn.Conv2d):
            units.append(Unit(m, mods[i + 1], (ACT_NONE, 1.0)))
            i += 2
        else:
            units.append(Unit(m, None, (ACT_NONE, 1.0)))
            i += 1
    return units


class Block:
    def __init__(self, blk):
        from ..models.resnet import BottleNeck
        self.units = _chain(blk.residual_function)
        sc = _chain(blk.shortcut) if len(blk.shortcut) > 0 else []
        assert len(sc) <= 1
        self.shortcut = sc[0] if sc else None
        self.join = (ACT_RELU, 1.0) if isinstance(blk, BottleNeck) else (ACT_CELU, 0.075)


STAGES = ("conv2_x", "conv3_x", "conv4_x", "conv5_x")

# The flat optimizer writes the packed conv weight layouts itself (optim_pack.hip: one fused
# update-and-pack launch) when the model's weights live in its flat buffer; the forward then
# skips its repack while nothing else has written the weights since (Plan.pack_fresh)
PACK_IN_OPT = os.environ.get("FDT_PACK_IN_OPT", "0") == "1"


class Plan:
    def __init__(self, model):
        stem_seq = model.conv1
        self.stem = Unit(stem_seq[0], None, _act_of(stem_seq[1]))
        self.blocks, self.stage_of = [], []
        for name in STAGES:
            for b in getattr(model, name):
                self.blocks.append(Block(b))
                self.stage_of.append(name)
        self.units = [self.stem] + [u for b in self.blocks for u in (b.units + ([b.shortcut] if b.shortcut else []))]
        self.fsdp = None  # parallel/fsdp.py FullyShardedDP driving the stages as wrap units

    def pack(self, dev, need_dgrad=True):
        if self.pack_fresh():
            return  # the optimizer's fused step already wrote both layouts from these weights
        ents = []
        for u in self.units:
            had = (u.wf, u.wd)
            u.ensure_packed_buffers(dev, need_dgrad and u is not self.stem)
            if u.wf is not had[0] or u.wd is not had[1]:
                self.__dict__.pop("_upd", None)  # the optimizer's table points at the old buffers
            ents.append((u.w.detach(), u.wf, u.wd, u.shp))
        ci.pack_weights(ents)

    # ---- packed layouts written by the optimizer (optim_pack.hip)
    def _weights_version(self, flat):
        # torch in-place writes (load_state_dict, copy_ into the flat buffer or a parameter) bump
        # these counters; the native optimizer kernels do not
        return flat.data._version + sum(u.w._version for u in self.units)

    def update_table(self, flat):
        """Launches of the fused update-and-pack step over ``flat`` (a FlatParams holding every
        conv weight as a contiguous fp32 OIHW view): a list of (entries int64 [n, 8], n, conv
        blocks, rest ranges int64 [m, 3], m, rest elements, max taps, counts a skipped step) --
        the 1x1 weights with every non-conv range at a 4 KB LDS image, then the 3x3 / 2x2
        weights at 38 KB -- or None when the layouts are not allocated yet (before the first
        training forward) or the weights are not all in ``flat``."""
        if not PACK_IN_OPT or self.fsdp is not None or not flat.data.is_cuda:
            return None
        c = self.__dict__.get("_upd")
        if c is not None and c[0] is flat:
            return c[1]
        if any(u.wf is None or (u.wd is None and u.shp.cin >= 8) for u in self.units):
            return None
        base, n = flat.data.data_ptr(), flat.numel
        rows = {1: [], 9: []}
        blks = {1: 0, 9: 0}
        spans = []
        for u in self.units:
            w = u.w
            off, rem = divmod(w.data_ptr() - base, 4)
            if (w.dtype != torch.float32 or not w.is_contiguous() or rem or off < 0 or off + w.numel() > n
                    or w.device != flat.data.device or w.dim() != 4):
                return None
            co, cin, kh, kw = w.shape
            if kh * kw not in (1, 4, 9) or co % 8 or u.shp.cxp % 8 or u.wf.device != w.device:
                return None
            g = 1 if kh * kw == 1 else 9
            rows[g].append([off, u.wf.data_ptr(), 0 if u.wd is None else u.wd.data_ptr(), co, cin, u.shp.cxp,
                            kh * kw, blks[g]])
            blks[g] += -(-co // 32) * -(-u.shp.cxp // 64)
            spans.append((off, off + w.numel()))
        spans.sort()
        rr, cur, cum = [], 0, 0
        for a, b in spans:
            if a < cur:
                return None  # overlapping weights
            if a > cur:
                rr.append([cur, a - cur, cum])
                cum += a - cur
            cur = b
        if cur < n:
            rr.append([cur, n - cur, cum])
            cum += n - cur
        dev = flat.data.device
        keep, launches = [], []
        for g in (1, 9):
            with_rest = g == 1
            if not rows[g] and not (with_rest and cum):
                continue
            tab = torch.tensor(rows[g] or [[0] * 8], dtype=torch.int64, device=dev)
            rrt = torch.tensor(rr or [[0, 0, 0]], dtype=torch.int64, device=dev)
            keep += [tab, rrt]
            launches.append((tab.data_ptr() if rows[g] else 0, len(rows[g]), blks[g],
                             rrt.data_ptr() if with_rest and rr else 0, len(rr) if with_rest else 0,
                             cum if with_rest else 0, g, int(not launches)))
        self._upd = (flat, launches, keep)
        # generation of the table: an NGD graph captured with the fused repack baked in the
        # table / layout addresses keys on it (optim/ngd.py _graph_key) -- a rebuilt table (new
        # packed buffers) never replays a graph holding the old, freed ones
        self.upd_gen = getattr(self, "upd_gen", 0) + 1
        return launches

    def mark_opt_packed(self, flat):
        """The optimizer step just written (or, when skipped on the device, left unchanged) the
        weights together with both packed layouts."""
        self._pk = (flat, self._weights_version(flat))

    def invalidate_pack(self):
        self.__dict__.pop("_pk", None)

    def pack_fresh(self) -> bool:
        pk = self.__dict__.get("_pk")
        return pk is not None and pk[1] == self._weights_version(pk[0])

    # ---- FSDP: units are gathered stage by stage, so weights are packed per stage (the
    # forward layout before the stage's forward, the dgrad layout before its backward) and
    # the packed copies are released with the gathered parameters
    # ---- lazy statistics: which units leave their statistics to the consumer, and where
    def lazy_layout(self, shape, dev):
        """{id(unit): (offset, rows)} of the lazy units for an input of ``shape`` (NHWC) and the
        zeroed slot arena they accumulate into (one arena per input shape: a captured graph's
        addresses never move; zeroed at every forward, inside the captured graph)."""
        if not lazy_enabled():
            return {}, None
        N, H, W = int(shape[0]), int(shape[1]), int(shape[2])
        key = (N, H, W, str(dev))
        cache = self.__dict__.setdefault("_lazy", {})
        ent = cache.get(key)
        if ent is None:
            offs, tot = {}, 0

            def add(u, h, w, conv_consumer=False):
                nonlocal tot
                ho, wo = ci.out_hw(h, w, u.shp)
                r = lazy_rows(N * ho * wo)
                # FusedConvBN units (mode 0) only: nn.BatchNorm2d units keep the standalone finalize
                # (running statistics, affine)
                if (u.bn is None and r * u.shp.cout <= LAZY_BUDGET and N * ho * wo > 1
                        and (LAZY_SCOPE == "all" or not conv_consumer)):
                    offs[id(u)] = (tot, r)
                    tot += (r * 2 + 4) * u.shp.cout  # slots | s | t | mean | sd
                return ho, wo

            h, w = add(self.stem, H, W)
            for bi, b in enumerate(self.blocks):
                hin, win = h, w
                nxt = self.blocks[bi + 1] if bi + 1 < len(self.blocks) else None
                ho_, wo_ = h, w
                for u in b.units:
                    ho_, wo_ = ci.out_hw(ho_, wo_, u.shp)
                folded = (nxt is not None and b.join[0] == ACT_RELU
                          and _join_fold_tile(nxt, (N, ho_, wo_)) is not None)
                for i, u in enumerate(b.units):
                    if i + 1 < len(b.units):
                        v = b.units[i + 1]  # consumer: a conv prologue unless a materialised 3x3
                        cc = not (MATERIALIZE_3X3 and v.shp.k > 1)
                    else:
                        cc = folded  # the join: a pass, or the next block's first conv (PRO_JOIN)
                    h, w = add(u, h, w, cc)
                if b.shortcut is not None:
                    add(b.shortcut, hin, win, folded)
            arena = torch.zeros(max(tot, 1), device=dev, dtype=torch.float32)
            ent = cache[key] = (offs, arena, tot)
        offs, arena, tot = ent
        if tot:
            arena[:tot].zero_()
        return offs, arena

    def stage_units(self, name):
        if name == "conv1":
            return [self.stem]
        return [u for b, st in zip(self.blocks, self.stage_of) if st == name
                for u in (b.units + ([b.shortcut] if b.shortcut else []))]

    def pack_stage(self, name, dev, fwd: bool):
        ents = []
        for u in self.stage_units(name):
            need_wd = (not fwd) and u is not self.stem
            u.ensure_packed_buffers(dev, need_wd)
            _restore(u.wf if fwd else u.wd)
            if fwd or need_wd:
                ents.append((u.w.detach(), u.wf if fwd else None, None if fwd else u.wd, u.shp))
        ci.pack_weights(ents)

    def release_stage(self, name, fwd: bool):
        if self.fsdp is not None and self.fsdp.static:
            return  # static FSDP (graphs): packed layouts keep their addresses
        for u in self.stage_units(name):
            _release(u.wf if fwd else u.wd)


def _release(t):
    if t is not None and t.untyped_storage().size() != 0:
        t.untyped_storage().resize_(0)


def _restore(t):
    if t is not None and t.untyped_storage().size() == 0:
        t.untyped_storage().resize_(t.numel() * t.element_size())


# ------------------------------------------------------------------ kernels glue
_SLOTS: dict = {}


def slots(nq, C, dev, M, wide=False):
    """The persistent statistics-slot workspace viewed as [rows, nq, C] for a producer over
    M output rows (rows = 64, more for a large-M 3x3 conv (``wide``), or one per workgroup in
    deterministic mode: ci.slot_rows).
    Producers (conv epilogues, BN-backward reductions) add into it with fp32 atomics; the
    consuming finalize / reduce kernel sums it in fp64 and re-zeroes it, so the next
    producer needs no memset.  One workspace suffices: every producer is consumed before
    the next one (and a view only ever covers rows its finalize re-zeroes)."""
    rows = ci.slot_rows(M, wide)
    n = max(ci.STAT_SLOTS * 3 * 2048, rows * nq * C)
    ws = _SLOTS.get(dev)
    if ws is None or ws.numel() < n:
        # (allocation happens in the eager warm-up step, before any graph capture)
        ws = torch.zeros(n, device=dev, dtype=torch.float32)
        _SLOTS[dev] = ws
    return ws[: rows * nq * C].view(rows, nq, C)


def _bn_fin_params(u: Unit, training):
    bn = u.bn
    mode = u.mode(training)
    if bn is not None:
        mom = bn.momentum if bn.momentum is not None else 0.1
        track = training and bn.track_running_stats
        rm = bn.running_mean if (track or mode == MODE_BN_EVAL) else None
        rv = bn.running_var if (track or mode == MODE_BN_EVAL) else None
        nbt = bn.num_batches_tracked if track else None
        return mode, mom, rm, rv, nbt, bn.weight, bn.bias
    return mode, 0.0, None, None, None, None, None


def lazy_enabled() -> bool:
    return LAZY_STATS and not _native.deterministic() and hasattr(_native.native(), "act_affine_lazy")


def lazy_rows(M: int) -> int:
    """Slot rows of a lazy producer over M output rows: one per 32 row blocks of the smallest
    (64-row) tile, a power of two <= 64."""
    nb = -(-int(M) // 64)
    r = 1
    while r * 32 < nb and r < 64:
        r *= 2
    return r


def _out_stats(u: Unit, M, training, dev, lay):
    """(statistics outputs (s, t, save_mean, save_aux), slot view, standalone-finalize args
    or None, lazy descriptor or None) of one unit's conv.  A lazy unit's outputs are views of
    its arena region (bn_math.h LazyStats layout), written by its consumer."""
    ent = lay[0].get(id(u)) if lay is not None else None
    if ent is None:
        st, fin = _fin_args(u, M, training, dev)
        return st, slots(2, u.shp.cout, dev, M, u.shp.k > 1), fin, None
    off, rows = ent
    C = u.shp.cout
    reg = lay[1][off:off + (rows * 2 + 4) * C]
    part = reg[:rows * 2 * C].view(rows, 2, C)
    outs = reg[rows * 2 * C:].view(4, C)
    st = (outs[0], outs[1], outs[2], outs[3])
    return st, part, None, ([reg.data_ptr()], [float(rows), float(u.eps), float(M)])


def conv_bn_fwd(x, u: Unit, s, t, act, training, dev, lazy_in=None, lay=None):
    """One unit's conv + batch statistics -> (y, (s, t, save_mean, save_aux), M, lazy).
    ``lazy_in``: the input's statistics are finalised in this conv's prologue; ``lazy`` (not
    None): this unit's own are left in the slot arena for its consumer (``Plan.lazy_layout``),
    otherwise a standalone finalize follows the conv."""
    Ho, Wo = ci.out_hw(x.shape[1], x.shape[2], u.shp)
    M = x.shape[0] * Ho * Wo
    st, part, fin, lz = _out_stats(u, M, training, dev, lay)
    y, _ = ci.conv_fwd(x, u.wf, u.shp, s, t, act[0] if act else 0, act[1] if act else 1.0,
                       part=part, fin=fin, lazy=lazy_in)
    return y, st, M, lz


def conv_bn_fwd_join(pj, u: Unit, training, dev, lay=None, tile=None):
    """``conv_bn_fwd`` of a block's first (1x1) unit whose input is the PREVIOUS block's
    join, computed in the conv's operand staging (ci.conv_fwd_join); the join output (this
    block's x_in) and its ReLU mask are stored on the way.  pj = (y, s, t, r, s2, t2, out,
    mask, lazy, lazy2); ``tile``: _join_fold_tile's choice (None / "tuned": the tuned table)."""
    y, s, t, r, s2, t2, out, mask, lz1, lz2 = pj
    M = y.numel() // y.shape[-1]
    st, part, fin, lz = _out_stats(u, M, training, dev, lay)
    tile = None if tile == "tuned" else tile
    yo, _ = ci.conv_fwd_join(y, r, s, t, s2, t2, u.wf, u.shp, out, mask, part=part, fin=fin, tile=tile, lazy=lz1,
                             lazy2=lz2)
    return yo, st, M, lz


def _join_fold_tile(b_next, shape):
    """Tile of the next block's first 1x1 conv when it computes this block's join in its operand
    staging (PRO_JOIN), or None for a standalone join pass.  The fused kernel wins when ONE
    output-channel tile covers the conv (each joined row is then computed and stored once;
    with several column tiles every tile re-reads both join operands: 1.2-2x slower than
    conv + join pass) -- scripts/join_probe.py, profiles/r5/join_probe_*.txt:
      Cout 64  (stage 1): the tuned tile; batch 1024 475 -> 355 us, batch 128 50 -> 44 us
      Cout 128 (stage 2): 128x128x64 at >= 2^17 rows (242 -> 195 us), else 64x128x64 (31 -> 25 us
                          in isolation, yet the batch-128 step measured 0.2 % slower folded)
      Cout 256 (stage 3): 128x256x64 at >= 2^16 rows (133 -> 124 us); slower at batch 128.
    A shape with a conv_tuned.json "fwd3" entry (scripts/retune_graph.py) is folded at that
    entry ("tuned"); others past 64 channels only over >= JOIN_FOLD_MIN_M rows.  Whole step at
    batch 1024: 25.66 -> 25.33 ms (profiles/r5/joinfold_bs1024_*.json).  ``shape``: the join's
    NHWC shape."""
    u = b_next.units[0]
    N, H = int(shape[0]), int(shape[1])
    M = N * H * int(shape[2])
    if not (JOIN_FOLD and u.shp.k == 1 and u.shp.stride == 1 and u.shp.pad == 0 and u.shp.cin == u.shp.cxp
            and u.shp.cin >= 8 and u.shp.cout <= JOIN_FOLD_MAX):
        return None
    if u.shp.cout <= 64:
        return "tuned"
    if u.shp.cout > 256 or (u.shp.cout > 128 and M < (1 << 16)):
        return None
    if ci.tuned("fwd3", N, H, u.shp):
        return "tuned"
    if M < JOIN_FOLD_MIN_M:
        return None
    if u.shp.cout <= 128:
        return (128, 128, 64) if M >= (1 << 17) else (64, 128, 64)
    return (128, 256, 64)


def _fin_args(u: Unit, M, training, dev):
    """Outputs (s, t, save_mean, save_aux) and the finalisation arguments of one unit's
    statistics (eval-mode BN reads none of them but still re-zeroes the slots)."""
    C = u.shp.cout
    s, t, sm, sa = _f32(C, dev), _f32(C, dev), _f32(C, dev), _f32(C, dev)
    mode, mom, rm, rv, nbt, gamma, beta = _bn_fin_params(u, training)
    fptr = [_p(gamma), _p(beta), _p(rm), _p(rv), _p(nbt), s.data_ptr(), t.data_ptr(), sm.data_ptr(), sa.data_ptr()]
    return (s, t, sm, sa), (fptr, [float(mode), float(u.eps), float(mom), float(M)])


def reduce_parts(part, nq, C, dev):
    nat = _native.native()
    out = torch.empty(nq, C, device=dev, dtype=torch.float32)
    nat.reduce_partials(part.data_ptr(), part.shape[0], nq, C, out.data_ptr(), 1, _sp())
    return out


def _coef_args(u: Unit, sm, sa, M, training, dev):
    """Kernel arguments of one unit's BN-backward coefficients; allocates (alpha, beta)
    and the BN affine gradients (accumulated into the flat gradient buffer)."""
    C = u.shp.cout
    al, be = _f32(C, dev), _f32(C, dev)
    gamma = u.bn.weight if u.bn is not None else None
    gg = gb = None
    if u.bn is not None:
        for p in (u.bn.weight, u.bn.bias):
            if p.requires_grad and p.grad is None:
                p.grad = torch.zeros_like(p)
        gg = u.bn.weight.grad if u.bn.weight.requires_grad else None
        gb = u.bn.bias.grad if u.bn.bias.requires_grad else None
    args = [u.mode(training), float(u.eps), float(M), sm.data_ptr(), sa.data_ptr(), _p(gamma), al.data_ptr(),
            be.data_ptr(), _p(gg), _p(gb)]
    return args, (al, be)


_NO_UNIT = [0, 0.0, 1.0, 0, 0, 0, 0, 0, 0, 0]


def coef_args(ua, sta, ub=None, stb=None, training=True, dev=None):
    """BN-backward coefficient arguments of unit ``ua`` (rows (0, 1) of the dL/dy slots) and,
    with nq == 3, of the block's shortcut unit ``ub`` (rows (2, 1)); ``st*`` = (save_mean,
    save_aux, M).  Returns ((fptr, fval) for ci.conv_dgrad(coef=...) / the standalone
    kernel, (alpha_a, beta_a), (alpha_b, beta_b) or None)."""
    aa, ra = _coef_args(ua, sta[0], sta[1], sta[2], training, dev)
    if ub is not None:
        ab, rb = _coef_args(ub, stb[0], stb[1], stb[2], training, dev)
    else:
        ab, rb = _NO_UNIT, None
    fptr = list(aa[3:]) + list(ab[3:])
    fval = [float(aa[0]), float(aa[1]), float(aa[2]), float(ab[0]), float(ab[1]), float(ab[2])]
    return (fptr, fval), ra, rb


def coef_ready(*units):
    for u in units:
        if u is not None and u.bn is not None:
            grad_ready(u.bn.weight)
            grad_ready(u.bn.bias)


def bwd_finalize(part, nq, ua, sta, ub=None, stb=None, training=True, dev=None):
    """Statistics slots [S, nq, C] of dL/dy reductions -> BN-backward corrections in one
    standalone launch (the slots are re-zeroed).  Returns ((alpha_a, beta_a), (alpha_b,
    beta_b) or None)."""
    (fptr, fval), ra, rb = coef_args(ua, sta, ub, stb, training, dev)
    ci._finalize_standalone(_native.native(), 2, part, nq, ua.shp.cout, fptr, fval)
    coef_ready(ua, ub)
    return ra, rb


def wgrad_into(u: Unit, g, y, al, be, x, xs, xt, act, gs=None):
    if u.w.grad is None:
        u.w.grad = torch.zeros_like(u.w)
    ci.conv_wgrad(g, y, al, be, x, u.shp, u.w.grad, xs, xt, act[0], act[1], accumulate=True, gs=gs)
    grad_ready(u.w)


def _rows(t):
    return t.numel() // t.shape[-1]


# weight gradients on a second stream (a parallel branch of the captured backward graph): they
# depend only on operands the dgrad chain has already produced, and nothing on the chain reads
# them until the optimizer, so each one can run beside the next units' dgrad -> BN-backward
# finalize -> fold chain.  Measured SLOWER on MI355X: batch 128 5.37 -> 5.96-5.99 ms, batch 1024
# 24.93 -> 25.32 ms (profiles/r5/wgrad_branch_*.json) -- the ~50 cross-stream fork / join
# dependencies per replayed backward cost more than the overlap returns, and the concurrent
# weight-gradient grids take CUs from the critical-path chain.  Opt-in (FDT_WGRAD_BRANCH=1).
WGRAD_BRANCH = os.environ.get("FDT_WGRAD_BRANCH", "0") == "1"
WGRAD_BRANCH_KEEP = 8 << 30  # bytes of branch operands held before a full join


class _WgradBranch:
    """The weight-gradient branch of one backward.  Hazards: (1) every operand a branch kernel
    reads stays referenced until the main stream has joined the branch, so the allocator cannot
    hand its memory to a main-stream tensor while the branch still reads it; (2) the one
    in-place overwrite of a branch operand -- an identity block's g_pre, accumulated into by
    its first unit's dgrad (g_x aliases g_pre) -- waits for the event recorded after the wgrad
    that reads it (``guard`` / ``wait``)."""

    _streams: dict = {}

    def __init__(self, dev):
        s = _WgradBranch._streams.get(dev)
        if s is None:
            s = _WgradBranch._streams[dev] = torch.cuda.Stream(device=dev)
        self.s = s
        self.main = torch.cuda.current_stream(dev)
        self.keep = []
        self.kept = 0
        self.event = None
        self._seg = None

    @staticmethod
    def make(dev):
        if not (WGRAD_BRANCH and dev.type == "cuda"):
            return None
        return _WgradBranch(dev)

    def run(self, u, g, y, al, be, x, xs, xt, act, gs=None, guard=False):
        rec = _graphs.active()
        if rec is not None and (rec, len(rec.segments)) != self._seg:
            # a graph segment may end at a hook's cut: the branch forked in it rejoins first
            self._seg = (rec, len(rec.segments))
            rec.joiners.append(lambda b=self.s: torch.cuda.current_stream().wait_stream(b))
        self.s.wait_stream(self.main)
        key = self._key()
        with torch.cuda.stream(self.s):
            wgrad_into(u, g, y, al, be, x, xs, xt, act, gs=gs)
            # (a gradient hook inside may have cut the graph: the ended segment joined this
            # branch, which is no longer part of the capture -- nothing to record then)
            if guard and self._key() == key:
                ev = torch.cuda.Event()
                ev.record(self.s)
                self.event = (ev, key)
        ops = [t for t in (g, y, al, be, x, xs, xt, gs) if isinstance(t, torch.Tensor)]
        self.keep.append(ops)
        self.kept += sum(t.numel() * t.element_size() for t in ops)
        if self.kept > WGRAD_BRANCH_KEEP:
            self.join()

    @staticmethod
    def _key():
        rec = _graphs.active()
        return None if rec is None else (rec, len(rec.segments))

    def _stale(self):
        """Under a graph recording whose segment ended since the branch last forked: the
        segment end already joined the branch (its joiner), and an event from the ended
        capture would be a dependency on uncaptured work."""
        rec = _graphs.active()
        return rec is not None and (rec, len(rec.segments)) != self._seg

    def wait(self):
        """Main stream: after the guarded wgrad (before overwriting its operand in place) --
        unless a segment ended since it was recorded (the segment end joined the branch)."""
        if self.event is not None and self.event[1] == self._key():
            self.main.wait_event(self.event[0])
        self.event = None

    def join(self, keep=False):
        if not self._stale():
            self.main.wait_stream(self.s)
        if not keep:
            self.keep, self.kept, self.event = [], 0, None


_ACTIVE_BRANCH = None  # the weight-gradient branch of the backward in progress (grad_ready)


def _wgrad(br, *args, guard=False, **kw):
    if br is None:
        wgrad_into(*args, **kw)
    else:
        br.run(*args, guard=guard, **kw)


# CELU joins (BasicBlock, reference resnet.py:188-190): the backward takes act'(z) = exp(z/alpha)
# from the fp32 pre-activation z = y*s + t + shortcut, recomputed from the stored bf16 branch
# outputs exactly as the forward join formed it.  FDT_CELU_ZGRAD=0 restores the old derivative
# 1 + o/alpha from the bf16 join OUTPUT o, which is wrong below z ~ -0.3 (bf16 ulp of o / alpha ~
# 6.5e-3 against a derivative < 0.02) and sign-flipped for deeply negative z (o rounds below
# -alpha): the ResNet-18 convergence gap of round 5 (profiles/r6/convergence_ablation.txt).
CELU_ZGRAD = os.environ.get("FDT_CELU_ZGRAD", "1") == "1"


def _celu_jz(b, ys, sc, x_in):
    """[sa, ta, sb, tb, xid] of a CELU join's z-mode backward (None: ReLU join / disabled)."""
    if b.join[0] != ACT_CELU or not CELU_ZGRAD:
        return None
    return [ys[-1][1], ys[-1][2], sc[1] if sc else None, sc[2] if sc else None, None if sc else x_in]


# ------------------------------------------------------------------ autograd node
class ResNetBodyFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x_nhwc, plan: Plan, training: bool, need_grad: bool):
        nat = _native.native()
        dev = x_nhwc.device
        fs = plan.fsdp
        if fs is None:
            plan.pack(dev, need_dgrad=need_grad)
        else:
            fs.pre_forward("conv1")
            plan.pack_stage("conv1", dev, fwd=True)
        recs = []
        lay = plan.lazy_layout(x_nhwc.shape, dev)
        # stem: conv -> FCBN stats -> materialised CELU output
        st = plan.stem
        y0, (s0, t0, sm0, sa0), M0, lz0 = conv_bn_fwd(x_nhwc, st, None, None, None, training, dev, lay=lay)
        h = torch.empty_like(y0)
        if lz0 is not None:
            nat.act_affine_lazy(y0.data_ptr(), lz0[0], lz0[1], h.data_ptr(), M0, st.shp.cout, st.act_out[0],
                                float(st.act_out[1]), 1, _sp())
        else:
            nat.act_affine_fwd(y0.data_ptr(), s0.data_ptr(), t0.data_ptr(), h.data_ptr(), M0, st.shp.cout,
                               st.act_out[0], float(st.act_out[1]), 1, 1, _sp())
        stem_rec = (x_nhwc, y0, s0, t0, sm0, sa0)
        cur = "conv1"
        pending = None  # previous block's join, run inside this block's first conv
        pend_tile = None  # ... at this tile (_join_fold_tile)
        for bi, b in enumerate(plan.blocks):
            if fs is not None and plan.stage_of[bi] != cur:
                plan.release_stage(cur, fwd=True)
                fs.post_forward(cur)
                cur = plan.stage_of[bi]
                fs.pre_forward(cur)
                plan.pack_stage(cur, dev, fwd=True)
            x_in = h
            ys = []
            raw, s, t, act, lz = x_in, None, None, (ACT_NONE, 1.0), None
            for ui, u in enumerate(b.units):
                a_in = None
                if ui == 0 and pending is not None:
                    # writes x_in (= the previous block's output) while staging it
                    y, (su, tu, smu, sau), M, lzo = conv_bn_fwd_join(pending, u, training, dev, lay, pend_tile)
                    pending = None
                elif MATERIALIZE_3X3 and u.shp.k > 1 and s is not None:
                    # 3x3: normalise + activate the input ONCE instead of in every one of the
                    # 9 im2col re-reads of the conv's operand staging (lazy statistics: the
                    # producer's finalize runs inside this pass)
                    a_in = torch.empty_like(raw)
                    if lz is not None:
                        nat.act_affine_lazy(raw.data_ptr(), lz[0], lz[1], a_in.data_ptr(), _rows(raw), raw.shape[-1],
                                            act[0], float(act[1]), 1, _sp())
                    else:
                        nat.act_affine_fwd(raw.data_ptr(), s.data_ptr(), t.data_ptr(), a_in.data_ptr(), _rows(raw),
                                           raw.shape[-1], act[0], float(act[1]), 1, 1, _sp())
                    y, (su, tu, smu, sau), M, lzo = conv_bn_fwd(a_in, u, None, None, None, training, dev, lay=lay)
                else:
                    y, (su, tu, smu, sau), M, lzo = conv_bn_fwd(raw, u, s, t, act, training, dev, lazy_in=lz,
                                                                lay=lay)
                ys.append((y, su, tu, smu, sau, M, a_in))
                raw, s, t, act, lz = y, su, tu, u.act_out, lzo
            y3, s3, t3, lz3 = ys[-1][0], ys[-1][1], ys[-1][2], lz
            sc, lzsc = None, None
            if b.shortcut is not None:
                u = b.shortcut
                ysc, (ssc, tsc, smsc, sasc), M, lzsc = conv_bn_fwd(x_in, u, None, None, None, training, dev, lay=lay)
                sc = (ysc, ssc, tsc, smsc, sasc, M, None)
            out = torch.empty_like(y3)
            C = y3.shape[-1]
            # ReLU joins also emit a 1-bit-per-element activation mask: the backward reads it
            # instead of `out` (1/16 of the bytes)
            mask = None
            if need_grad and b.join[0] == ACT_RELU:
                mask = torch.empty(out.numel() // 8, device=dev, dtype=torch.uint8)
            nxt = plan.blocks[bi + 1] if bi + 1 < len(plan.blocks) else None
            pend_tile = _join_fold_tile(nxt, y3.shape) if nxt is not None and b.join[0] == ACT_RELU else None
            if pend_tile is not None:
                # the next block's first 1x1 conv computes this join while staging its operand
                # and stores `out` + mask (one pass instead of join pass + operand re-read)
                pending = (y3, s3, t3, sc[0] if sc else x_in, sc[1] if sc else None, sc[2] if sc else None, out, mask,
                           lz3, lzsc)
            elif lz3 is not None:
                lzb = lzsc if lzsc is not None else ([], [])
                nat.residual_act_lazy(y3.data_ptr(), lz3[0], lz3[1], _p(sc[0] if sc else None), lzb[0], lzb[1],
                                      _p(sc[1] if sc and lzsc is None else None),
                                      _p(sc[2] if sc and lzsc is None else None), 0 if sc else x_in.data_ptr(),
                                      out.data_ptr(), _p(mask), _rows(y3), C, b.join[0], float(b.join[1]), 1, _sp())
            else:
                nat.residual_act_fwd(y3.data_ptr(), s3.data_ptr(), t3.data_ptr(), _p(sc[0] if sc else None),
                                     _p(sc[1] if sc else None), _p(sc[2] if sc else None),
                                     0 if sc else x_in.data_ptr(), out.data_ptr(), _p(mask), _rows(y3), C, b.join[0],
                                     float(b.join[1]), 1, _sp())
            if need_grad:
                recs.append((x_in, ys, sc, out, mask))
            h = out
        if fs is not None:
            plan.release_stage(cur, fwd=True)
            fs.post_forward(cur)
        head_rec = None
        if getattr(plan, "head_on", False):
            h, head_rec = head_forward(plan.fc, h)
        if need_grad:
            ctx.plan, ctx.training = plan, training
            ctx.recs, ctx.stem_rec = recs, stem_rec
            ctx.head_rec = head_rec
        return h

    @staticmethod
    def backward(ctx, g_out):
        """Blocks in reverse order.  The gradient of a block's output arrives ALREADY through
        that block's join backward (g_pre = g*act'(out), plus its 3 statistics rows in the
        slot workspace): the next block's last dgrad -- the one that completes the gradient
        of its input -- ran the join backward in its epilogue (EPI_JOINBWD).  Only the last
        block (its gradient comes from the pooling) runs the standalone join kernel.
        Within a block the shortcut dgrad goes first (a full-coverage store of the input
        gradient; a strided shortcut writes its zero parity classes too) so the final writer
        is always the stride-1 first unit."""
        nat = _native.native()
        plan, training = ctx.plan, ctx.training
        ghw = 0  # > 0: g is the head's pooled gradient, broadcast over ghw rows per sample
        if getattr(ctx, "head_rec", None) is not None:
            g, ghw = head_backward(plan.fc, g_out, ctx.head_rec)
        else:
            g = g_out.contiguous()
        dev = g.device
        recs = ctx.recs
        nblk = len(plan.blocks)
        fs = plan.fsdp
        global _ACTIVE_BRANCH
        br = _ACTIVE_BRANCH = _WgradBranch.make(dev)
        try:
            return ResNetBodyFn._backward_blocks(ctx, plan, training, g, ghw, dev, recs, nblk, fs, br)
        finally:
            _ACTIVE_BRANCH = None

    @staticmethod
    def _backward_blocks(ctx, plan, training, g, ghw, dev, recs, nblk, fs, br):
        nat = _native.native()
        joined = False  # g is already g_pre of the current block (its BN-backward coefficients
        joined_coef = None  # computed with the dgrad that completed it: joined_coef)
        cur = None
        for bi in range(nblk - 1, -1, -1):
            b = plan.blocks[bi]
            if fs is not None and plan.stage_of[bi] != cur:
                if cur is not None:
                    if br is not None:
                        br.join()  # the stage's gradients are complete before its reduce-scatter
                    plan.release_stage(cur, fwd=False)
                    fs.post_backward(cur)
                cur = plan.stage_of[bi]
                fs.pre_backward(cur)
                plan.pack_stage(cur, dev, fwd=False)
            x_in, ys, sc, out, mask = recs[bi]
            y3, s3 = ys[-1][0], ys[-1][1]
            C = y3.shape[-1]
            M = _rows(y3)
            part = slots(3, C, dev, M)
            if joined:
                gpre = g
            else:
                # ONE gradient g_pre = g*act'(z) for both branches: each consumer folds in its
                # own BN scale (gs = s3 / s_shortcut) in its prologue
                gpre = torch.empty_like(y3)
                jz = _celu_jz(b, ys, sc, x_in)
                nat.residual_act_bwd(g.data_ptr(), 0 if (mask is not None or jz) else out.data_ptr(), _p(mask),
                                     y3.data_ptr(), _p(sc[0] if sc else None), gpre.data_ptr(), part.data_ptr(),
                                     part.shape[0], M, C,
                                     b.join[0], float(b.join[1]), 1, _sp(), ghw, [_p(v) for v in jz] if jz else [])
                ghw = 0
            ul = b.units[-1]
            if joined:
                (al, be), coef_sc = joined_coef  # finalised with the completing dgrad (below)
            else:
                (al, be), coef_sc = bwd_finalize(part, 3, ul, (ys[-1][3], ys[-1][4], ys[-1][5]),
                                                 b.shortcut, (sc[3], sc[4], sc[5]) if sc else None, training, dev)
            assert sc is not None or len(b.units) > 1, "identity block needs >1 unit (g_pre aliasing)"
            if sc is not None:
                u = b.shortcut
                als, bes = coef_sc
                g_x, _ = ci.conv_dgrad(gpre, sc[0], als, bes, u.wd, u.shp, tuple(x_in.shape), epi=ci.EPI_STORE,
                                       gs=sc[1])
                _wgrad(br, u, gpre, sc[0], als, bes, x_in, None, None, (ACT_NONE, 1.0), gs=sc[1])
            else:
                g_x = gpre  # identity: the x_in gradient accumulates onto g_pre in place
            # the block whose output is x_in: its join backward runs in the epilogue of the
            # dgrad that completes g_x (unit 0's, below) when that dgrad is dense (a strided
            # unit 0 -- BasicBlock downsampling -- writes parity classes: standalone join)
            prev = plan.blocks[bi - 1] if (bi > 0 and b.units[0].shp.stride == 1) else None
            prec = recs[bi - 1] if bi > 0 else None
            g_cur, gs_cur = gpre, s3
            # residual chain, last unit first; (al, be) = BN-backward correction of unit i
            for i in range(len(b.units) - 1, -1, -1):
                u = b.units[i]
                y, su, tu, smu, sau, Mu, a_in = ys[i]
                if i > 0:
                    yp, sp_, tp = ys[i - 1][0], ys[i - 1][1], ys[i - 1][2]
                    actp = b.units[i - 1].act_out
                    pp = slots(2, u.shp.cin, dev, _rows(yp), u.shp.k > 1)
                    up = b.units[i - 1]
                    cf, (al_p, be_p), _ = coef_args(up, (ys[i - 1][3], ys[i - 1][4], ys[i - 1][5]),
                                                    training=training, dev=dev)
                    if MATERIALIZE_3X3 and u.shp.k > 1:
                        # fold the BN-backward correction into the gradient once (3x3: the
                        # dgrad operand is re-read 9x, the wgrad operand once per column block)
                        gf = torch.empty_like(g_cur)
                        nat.affine_fold(g_cur.data_ptr(), y.data_ptr(), al.data_ptr(), be.data_ptr(), _p(gs_cur),
                                        gf.data_ptr(), _rows(gf), gf.shape[-1], 1, _sp())
                        g_prev, _ = ci.conv_dgrad(gf, None, None, None, u.wd, u.shp, tuple(yp.shape),
                                                  epi=ci.EPI_ACTBWD, ex=yp, es=sp_, et=tp, act=actp[0],
                                                  alpha=actp[1], part=pp, coef=cf)
                        _wgrad(br, u, gf, None, None, None, a_in if a_in is not None else yp,
                               None if a_in is not None else sp_, None if a_in is not None else tp,
                               (ACT_NONE, 1.0) if a_in is not None else actp)
                    else:
                        g_prev, _ = ci.conv_dgrad(g_cur, y, al, be, u.wd, u.shp, tuple(yp.shape),
                                                  epi=ci.EPI_ACTBWD, ex=yp, es=sp_, et=tp, act=actp[0],
                                                  alpha=actp[1], part=pp, gs=gs_cur, coef=cf)
                        # (the last unit reads g_pre: an identity block's first-unit dgrad
                        # later accumulates into it in place -- guarded)
                        _wgrad(br, u, g_cur, y, al, be, yp, sp_, tp, actp, gs=gs_cur,
                               guard=(i == len(b.units) - 1 and sc is None))
                    coef_ready(up)
                    al, be = al_p, be_p
                    g_cur, gs_cur = g_prev, None
                else:
                    if br is not None and sc is None:
                        br.wait()  # g_x aliases g_pre: its last reader (a branch wgrad) first
                    if prev is not None:
                        px_in, pys, psc, pout, pmask = prec
                        pjz = _celu_jz(prev, pys, psc, px_in)
                        pul = prev.units[-1]
                        cf, ra, rb = coef_args(pul, (pys[-1][3], pys[-1][4], pys[-1][5]), prev.shortcut,
                                               (psc[3], psc[4], psc[5]) if psc else None, training, dev)
                        ci.conv_dgrad(g_cur, y, al, be, u.wd, u.shp, tuple(x_in.shape), epi=ci.EPI_JOINBWD, out=g_x,
                                      gs=gs_cur, ex=pys[-1][0], part=slots(3, x_in.shape[-1], dev, _rows(x_in)),
                                      act=prev.join[0], alpha=prev.join[1], jmask=pmask,
                                      jyb=psc[0] if psc else None,
                                      jout=None if (pmask is not None or pjz) else pout, coef=cf,
                                      es=pjz[0] if pjz else None, et=pjz[1] if pjz else None,
                                      jz=pjz[2:] if pjz else None)
                        coef_ready(pul, prev.shortcut)
                        joined_coef = (ra, rb)
                    else:
                        ci.conv_dgrad(g_cur, y, al, be, u.wd, u.shp, tuple(x_in.shape), epi=ci.EPI_ADD, out=g_x,
                                      gs=gs_cur)
                    _wgrad(br, u, g_cur, y, al, be, x_in, None, None, (ACT_NONE, 1.0), gs=gs_cur)
            g = g_x
            joined = prev is not None
        if fs is not None and cur is not None:
            if br is not None:
                br.join()
            plan.release_stage(cur, fwd=False)
            fs.post_backward(cur)
            fs.pre_backward("conv1")
        # stem: act backward + statistics -> wgrad on the input image
        x_img, y0, s0, t0, sm0, sa0 = ctx.stem_rec
        st = plan.stem
        M0 = _rows(y0)
        C0 = st.shp.cout
        part = slots(2, C0, dev, M0)
        gy0 = torch.empty_like(y0)
        nat.act_bwd_reduce(g.data_ptr(), y0.data_ptr(), s0.data_ptr(), t0.data_ptr(), gy0.data_ptr(),
                           part.data_ptr(), part.shape[0], M0, C0, st.act_out[0], float(st.act_out[1]), 1, _sp())
        (al, be), _ = bwd_finalize(part, 2, st, (sm0, sa0, M0), training=training, dev=dev)
        _wgrad(br, st, gy0, y0, al, be, x_img, None, None, (ACT_NONE, 1.0))
        if br is not None:
            br.join()
        if fs is not None:
            fs.post_backward("conv1")
        if not getattr(ctx, "keep", False):
            ctx.recs = ctx.stem_rec = ctx.head_rec = None
        return None, None, None, None


# ------------------------------------------------------------------ classifier head
def head_fusable(model, x, need_grad) -> bool:
    """The fused head reproduces ``fc(mean_hw(body))`` under bf16 autocast for heads of at
    most 32 classes with fp32 parameters / gradients; anything else keeps the PyTorch ops."""
    fc = getattr(model, "fc", None)
    if not FUSED_HEAD or not getattr(model, "fused_head", True) or not isinstance(fc, nn.Linear) or fc.bias is None or getattr(model, "_fsdp", None) is not None:
        return False
    if not isinstance(getattr(model, "avg_pool", None), nn.AdaptiveAvgPool2d) or fc._forward_hooks or fc._forward_pre_hooks:
        return False
    dt = x.device.type
    if not (torch.is_autocast_enabled(dt) and torch.get_autocast_dtype(dt) == BF16):
        return False
    if not hasattr(_native.native(), "head_fwd"):
        return False
    K, C = fc.weight.shape
    if K > 32 or C % 8:
        return False
    for p in (fc.weight, fc.bias):
        if p.dtype != torch.float32 or not p.is_contiguous() or (need_grad and not p.requires_grad):
            return False
        if p.grad is not None and (p.grad.dtype != torch.float32 or not p.grad.is_contiguous()):
            return False
    return True


def head_forward(fc, h):
    """body [N,H,W,C] bf16 -> (logits [N,K] bf16, (pooled bf16 [N,C], H*W))."""
    N, H, W, C = h.shape
    K = fc.weight.shape[0]
    pooled = torch.empty(N, C, device=h.device, dtype=BF16)
    logits = torch.empty(N, K, device=h.device, dtype=BF16)
    _native.native().head_fwd(h.data_ptr(), fc.weight.data_ptr(), fc.bias.data_ptr(), pooled.data_ptr(),
                              logits.data_ptr(), N, H * W, C, K, _sp())
    return logits, (pooled, H * W)


def head_backward(fc, g_logits, rec):
    """Accumulates fc.weight.grad / fc.bias.grad (signalling their readiness) and returns
    the pooled gradient [N,C] bf16 (already / HW) with its broadcast row count HW."""
    pooled, hw = rec
    N, C = pooled.shape
    K = fc.weight.shape[0]
    dl = g_logits.to(BF16).contiguous()
    for p in (fc.weight, fc.bias):
        if p.grad is None:
            p.grad = torch.zeros_like(p)
    dpool = torch.empty(N, C, device=pooled.device, dtype=BF16)
    _native.native().head_bwd(dl.data_ptr(), fc.weight.data_ptr(), pooled.data_ptr(), dpool.data_ptr(),
                              fc.weight.grad.data_ptr(), fc.bias.grad.data_ptr(), N, hw, C, K, _sp())
    grad_ready(fc.bias)
    grad_ready(fc.weight)
    return dpool, hw


def to_engine_input(x: torch.Tensor, cxp: int = 8) -> torch.Tensor:
    """(N,3,H,W) image batch (any layout/dtype) -> (N,H,W,cxp) bf16 zero-padded NHWC.
    Zero-copy when x is the channel-sliced NCHW view of such a buffer (the device CIFAR
    loader produces exactly that)."""
    N, C, H, W = x.shape
    if x.dtype == BF16 and x.stride() == (H * W * cxp, 1, W * cxp, cxp):
        return torch.as_strided(x, (N, H, W, cxp), (H * W * cxp, W * cxp, cxp, 1))
    out = torch.zeros(N, H, W, cxp, device=x.device, dtype=BF16)
    out[..., :C] = x.permute(0, 2, 3, 1)
    return out


def resnet_engine_forward(model, x):
    """Forward of ``models.resnet.ResNet`` through the engine; returns logits."""
    plan = getattr(model, "_plan", None)
    if plan is None:
        plan = model._plan = Plan(model)
    plan.fsdp = getattr(model, "_fsdp", None)
    # FSDP: graph segments between the stages only in static mode (persistent buffers; the
    # collectives run as actions between segments); eager otherwise
    plan.use_graphs = bool(getattr(model, "graph_engine", False)) and (plan.fsdp is None or plan.fsdp.static)
    xin = to_engine_input(x, plan.stem.shp.cxp)
    need_grad = torch.is_grad_enabled() and any(p.requires_grad for p in model.parameters())
    plan.fc = model.fc
    plan.head_on = head_fusable(model, x, need_grad)
    if need_grad:
        # the engine writes weight gradients itself; autograd sees one node whose only
        # differentiable input is a dummy (the image batch needs no gradient)
        dummy = torch.empty(0, device=x.device, requires_grad=True)
        body = _BodyWithDummy.apply(xin, dummy, plan, model.training)
    else:
        body = ResNetBodyFn.forward(_NoCtx(), xin, plan, model.training, False)
    if plan.head_on:
        return body  # logits of the fused head
    pooled = body.mean(dim=(1, 2), dtype=torch.float32)  # fp32 accumulation, no fp32 copy of the body
    return model.fc(pooled)


class _NoCtx:
    pass


class _GraphState:
    """HIP graphs of one (batch shape, train/eval) configuration of the body.

    Step 1 runs eagerly (warm-up: lazy kernel attributes, slot workspace, allocator).
    Step 2 captures the forward into one graph and the backward into segments cut where a
    gradient bucket becomes ready, then replays them.  Later steps copy the batch into the
    static input, replay the forward graph, and in backward copy the incoming gradient and
    replay the segments, launching each bucket's all-reduce between them.  Every kernel of
    the body (~400 at ResNet-50) is then one graph launch per segment: the host no longer
    paces the GPU at small per-GPU batches (the 8-GPU case)."""

    def __init__(self):
        self.stage = "warm"
        self.pool = None
        self.x = self.h = self.g = None
        self.inner = None
        self.fwd = None
        self.segments = None
        self.repacks = True


def graphs_enabled(plan) -> bool:
    return getattr(plan, "use_graphs", False) and os.environ.get("FDT_GRAPHS", "1") != "0"


class _BodyWithDummy(torch.autograd.Function):
    """Gives the body node a differentiable input so autograd calls its backward even
    though the image batch does not require grad.  With graphs enabled the body runs as
    captured HIP graphs (see ``_GraphState``)."""

    @staticmethod
    def forward(ctx, xin, dummy, plan, training):
        st = None
        if graphs_enabled(plan):
            key = (tuple(xin.shape), bool(training), bool(getattr(plan, "head_on", False)))
            states = plan.__dict__.setdefault("_graphs", {})
            st = states.get(key)
            if st is None:
                states[key] = _GraphState()  # this step: eager warm-up
            elif st.stage == "warm":
                st.pool = torch.cuda.graph_pool_handle()
                st.x = xin.clone()
                st.inner = _NoCtx()
                st.inner.keep = True
                # forward as graph segments: one, or (static FSDP) one per stage with each
                # unit's all-gather wait / next-unit prefetch as actions between them
                cur = torch.cuda.current_stream()
                side = torch.cuda.Stream()
                side.wait_stream(cur)
                torch.cuda.synchronize()
                rec = _graphs.Recorder(st.pool)
                st.repacks = not plan.pack_fresh()  # does the captured forward repack the weights?
                with torch.cuda.stream(side), _graphs.recording(rec), _graphs.capture_guard():
                    rec.begin()
                    try:
                        st.h = ResNetBodyFn.forward(st.inner, st.x, plan, training, True)
                    finally:
                        rec.end()
                cur.wait_stream(side)
                st.fwd = rec
                st.fwd.replay()
                st.stage = "fwd"
            else:
                if not st.repacks and not plan.pack_fresh():
                    # captured without the repack (the optimizer packs): weights written since by
                    # something else -- repack before the replay
                    plan.pack(xin.device, need_dgrad=True)
                st.x.copy_(xin)
                st.fwd.replay()
        ctx.gstate = st if (st is not None and st.stage in ("fwd", "ready")) else None
        if ctx.gstate is not None:
            return st.h.detach()
        ctx.inner = _NoCtx()
        return ResNetBodyFn.forward(ctx.inner, xin, plan, training, True)

    @staticmethod
    def backward(ctx, g):
        st = ctx.gstate
        if st is None:
            ResNetBodyFn.backward(ctx.inner, g)
            return None, None, None, None
        if st.stage == "fwd":
            st.g = g.detach().clone().contiguous()
            side = torch.cuda.Stream()
            side.wait_stream(torch.cuda.current_stream())
            torch.cuda.synchronize()
            rec = _graphs.Recorder(st.pool)
            with torch.cuda.stream(side), _graphs.recording(rec), _graphs.capture_guard():
                rec.begin()
                try:
                    ResNetBodyFn.backward(st.inner, st.g)
                finally:
                    rec.end()
            torch.cuda.current_stream().wait_stream(side)
            st.rec = rec
            st.segments = rec.segments
            st.stage = "ready"
        else:
            st.g.copy_(g)
        st.rec.replay()
        if st.rec.needs_check:
            # first replay of a backward whose bucket all-reduces were captured in-graph:
            # checked against eager all-reduces (parallel/graphs.py); the checking graph (it
            # snapshots every bucket) is dropped and the next step recaptures the backward --
            # in capture mode, or with cuts if the check failed
            st.rec.check_collectives()
            st.stage, st.rec, st.segments = "fwd", None, None
        return None, None, None, None
