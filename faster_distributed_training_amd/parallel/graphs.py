"""HIP-graph capture of a training step whose backward launches DDP bucket all-reduces.

A replayed HIP graph runs no Python, so the reducer's hooks cannot launch a bucket's
collective in the middle of a replay.  Instead the capture is CUT where a bucket completes
(the reducer's hook calls ``Recorder.cut`` with the launch as a deferred action): the step
becomes graph segments, and a replay runs ``segment, its bucket launches, next segment,
...`` -- every collective still starts as soon as its gradients are final and overlaps the
rest of backward, while the host issues one graph launch per segment instead of hundreds
of kernels (the transformer at 32 samples/GPU is host-bound without graphs).

Used by the fused ResNet engine (ops/resnet_fused.py: backward captured inside its
autograd node) and by ``SegmentedStep`` (any forward + autograd backward, e.g. the
transformer trainer under DDP; its backward capture starts in the loss's backward node so
that it runs on autograd's device thread like the hooks that cut it).  Reference: DDP's bucketed overlap
(``resnet50_test.py:716``, ``transformer_test.py:241-271``).
"""
from __future__ import annotations

import contextlib
import os

import time

import torch
from torch.utils._python_dispatch import TorchDispatchMode

# The recorder of the capture in progress (read by parallel/ddp.py hooks and the engine's
# grad_ready from the autograd thread); None outside a capture.
_ACTIVE = None

# How DETACHED actions are placed -- collectives that nothing later in the graph reads
# (DDP / ZeRO bucket all-reduces; the compute stream meets them only after the step's backward):
#   "capture": the capture is NOT cut.  The action runs INSIDE the capture, from a side stream
#            forked off the capture stream at that point, so the collective (RCCL) becomes a
#            node on a side branch of the backward graph; the branch is joined into the capture
#            stream only where the segment ends.  HIP graph replays run forked branches
#            concurrently (measured: two 1 ms branches replay in 1.03 ms,
#            profiles/r4/graph_comm_probe.txt), so the all-reduce overlaps the rest of backward
#            while the backward stays ONE graph -- no graph-boundary bubbles on the compute queue.
#            Needs a capturable backend (nccl = RCCL); with gloo the action falls back to a cut.
#   "cut":   the capture is cut there and the action runs between the two replayed segments
#            (round-3 scheme: ~25-50 us of compute-queue idle per cut, profiles/r3s3/).
# (An external event-record node, the CUDA idiom for "start this stream mid-graph", is refused
# by torch on ROCm: "External events are disallowed in rocm".)
#
# FDT_GRAPH_COMM selects: "auto" (default) = "capture", CHECKED IN-RUN: the first backward captured
# with collectives inside also snapshots every bucket right before its in-graph all-reduce; after
# that graph's first replay each bucket's in-graph result is compared with an eager all-reduce of
# its snapshot (same data, same group).  Equal: the process keeps capture mode (the checking graph
# is dropped and the backward recaptured without snapshots).  Different on any rank: the step's
# buckets are overwritten with the eager results, the process switches to "cut" for the rest of
# the run (no restart: the owner just recaptures) and ``STATUS`` says "cut(fallback)" -- bench.py
# reports it as ``graph_comm``.  "capture" = capture unchecked, "cut" = always cut.
_REQUESTED = os.environ.get("FDT_GRAPH_COMM", "auto")
DETACHED_MODE = "cut" if _REQUESTED == "cut" else "capture"
CHECK = _REQUESTED == "auto"
# "unchecked" until the check ran; then "capture" | "capture(order-tolerant)" | "cut(fallback)";
# "cut" / "capture(unchecked)" when FDT_GRAPH_COMM forces a mode
STATUS = {"auto": "unchecked", "capture": "capture(unchecked)"}.get(_REQUESTED, "cut")
# test hook (tests/test_distributed_gpu.py): the captured join of every bucket corrupts its
# all-reduced buffer, as a broken in-graph collective would -- the check must fall back
CORRUPT_FOR_TEST = os.environ.get("FDT_GRAPH_COMM_CORRUPT", "0") == "1"


def comm_status():
    """What the detached collectives of this process do now (bench JSON ``graph_comm``)."""
    return STATUS if DETACHED_MODE == "capture" or STATUS == "cut(fallback)" else "cut"


def checking():
    """True while the in-graph collective check is still to be done in this process."""
    return CHECK and DETACHED_MODE == "capture" and STATUS == "unchecked"


def reset_check(requested: str = "auto"):
    """(tests) re-arm the mode selection as if FDT_GRAPH_COMM were ``requested``."""
    global DETACHED_MODE, CHECK, STATUS
    DETACHED_MODE = "cut" if requested == "cut" else "capture"
    CHECK = requested == "auto"
    STATUS = {"auto": "unchecked", "capture": "capture(unchecked)"}.get(requested, "cut")


def active():
    return _ACTIVE


def detached(fn, capturable=False):
    """Mark ``fn`` (a deferred GPU action) as one nothing in the captured graph reads.
    ``capturable``: ``fn`` may run inside the capture (a RCCL collective) and returns a
    joiner -- a callable that orders its completion into the current stream."""
    fn.detached = True
    fn.capturable = bool(capturable)
    return fn


_COMM_SIDE = {}


def _comm_side_stream(device):
    """Side stream the captured detached actions are issued from (high priority: in eager
    use it never shares the compute stream's hardware queue)."""
    idx = torch.device(device).index if torch.device(device).index is not None else torch.cuda.current_device()
    st = _COMM_SIDE.get(idx)
    if st is None:
        st = _COMM_SIDE[idx] = torch.cuda.Stream(device=idx, priority=-1)
    return st


def drain_comm_watch():
    """Finish every eager collective and give RCCL's watchdog thread a polling interval (100 ms)
    to retire them, before a capture that can take collectives.  The watchdog polls the
    completion event of every eager collective still on its list; once that collective's stream
    has joined a graph capture (the first captured collective makes it join), HIP refuses the
    query ("operation not permitted on an event last recorded in a capturing stream") and the
    watchdog aborts the process -- seen in the closing runs of rounds 5 and 6, in the
    capture-check test, whose eager check all-reduces are followed at once by the recapture."""
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()) or dist.get_backend() != "nccl":
        return
    torch.cuda.synchronize()
    time.sleep(0.25)


class Recorder:
    """Capture split into graph segments at deferred hook actions.

    Begin, cuts and end must all happen on ONE thread (HIP rejects ending a capture from
    another thread): autograd's device thread, where backward nodes and gradient hooks run.
    A cut ends and restarts the capture on the stream it began on, after joining the
    caller's current stream if autograd runs the hook on another (forked, captured) one."""

    def __init__(self, pool, mode="thread_local"):
        self.pool = pool
        self.mode = mode
        self.segments = []  # [(CUDAGraph, [actions to run after it])]
        self.cur = None
        self.stream = None
        self.foreign_cuts = 0  # cuts requested from a stream other than the capture stream
        self.joiners = []      # captured detached actions of the open segment, joined at its end
        self.captured = 0      # detached actions captured on a side branch (no cut)
        # in-graph collective check (module docstring, FDT_GRAPH_COMM=auto): collectives captured
        # while ``checking`` register (snapshot, result buffer, op, group, fix) here
        self.checking = checking()
        self.checks = []

    def begin(self):
        if self.stream is None:
            # (autograd's device thread; the capture has not begun: synchronising is allowed)
            drain_comm_watch()
            self.stream = torch.cuda.current_stream()
        with torch.cuda.stream(self.stream):
            self.cur = torch.cuda.CUDAGraph()
            self.cur.capture_begin(pool=self.pool, capture_error_mode=self.mode)

    def _join(self):
        caller = torch.cuda.current_stream()
        if caller != self.stream:
            self.foreign_cuts += 1
            self.stream.wait_stream(caller)

    def cut(self, actions):
        self._join()
        if (DETACHED_MODE == "capture" and actions
                and all(getattr(a, "detached", False) and getattr(a, "capturable", False) for a in actions)):
            # no cut: fork a side branch here and run the collectives inside the capture
            side = _comm_side_stream(self.stream.device)
            side.wait_stream(self.stream)
            with torch.cuda.stream(side):
                for a in actions:
                    j = a()
                    if j is not None:
                        self.joiners.append(j)
            self.joiners.append(lambda s=side: torch.cuda.current_stream().wait_stream(s))
            self.captured += len(actions)
            return
        self._end_segment(actions)
        self.begin()

    def _end_segment(self, actions):
        with torch.cuda.stream(self.stream):
            for j in self.joiners:  # every side branch forked in this segment rejoins before its end
                j()
            self.joiners = []
            self.cur.capture_end()
        self.segments.append((self.cur, list(actions)))

    def end(self):
        self._join()
        self._end_segment([])
        self.cur = None

    def replay(self):
        for graph, acts in self.segments:
            graph.replay()
            for a in acts:
                a()

    @property
    def needs_check(self):
        return self.checking and bool(self.checks)

    def check_collectives(self):
        """After the FIRST replay of a checking capture: compare every captured collective's
        result with an eager all-reduce of its pre-collective snapshot.  Every rank runs the
        same checks in the same order (same capture), then agrees on the verdict (MAX).
        Returns True when capture mode stands; on a mismatch the buckets of this step get the
        eager results and the process falls back to cut mode.  Either way the caller drops
        this recorder's graphs and recaptures (without snapshots)."""
        global DETACHED_MODE, STATUS
        import torch.distributed as dist
        torch.cuda.current_stream().synchronize()
        worst, exact, pg = 0.0, True, None
        for shadow, buf, op, group, fix in self.checks:
            ref = shadow.clone()
            dist.all_reduce(ref, op=op, group=group)
            pg = group
            if not torch.equal(ref, buf):
                exact = False
                scale = float(ref.float().abs().max()) or 1.0
                worst = max(worst, float((ref.float() - buf.float()).abs().max()) / scale)
                fix(ref)
        verdict = torch.tensor([worst, 0.0 if exact else 1.0], dtype=torch.float64, device=self.stream.device)
        dist.all_reduce(verdict, op=dist.ReduceOp.MAX, group=pg)
        worst, inexact = float(verdict[0]), bool(verdict[1] > 0)
        self.checks = []
        self.checking = False
        # (a sum in another order differs in the last bits; a broken hand-off does not stop there)
        if not inexact:
            STATUS = "capture"
        elif worst <= 1e-5:
            STATUS = "capture(order-tolerant)"
        else:
            STATUS = "cut(fallback)"
            DETACHED_MODE = "cut"
            if dist.get_rank() == 0:
                print(f"[graphs] in-graph collectives disagree with eager all-reduce (max rel diff {worst:.3g}): "
                      f"falling back to graph cuts for this run", flush=True)
        return DETACHED_MODE == "capture"


class recording:
    """``with recording(rec):`` hooks that complete a DDP bucket cut ``rec`` instead of
    launching the collective."""

    def __init__(self, rec: Recorder):
        self.rec = rec

    def __enter__(self):
        global _ACTIVE
        assert _ACTIVE is None, "nested graph recordings"
        _ACTIVE = self.rec
        return self.rec

    def __exit__(self, *exc):
        global _ACTIVE
        _ACTIVE = None


class _BackwardCaptureStart(torch.autograd.Function):
    """Identity on the loss.  Its backward is the first node autograd runs, on its device
    thread: the backward capture begins there (HIP refuses to end or cut a capture from a
    thread other than the one that began it, and the bucket hooks cut from that thread);
    the capture ends in autograd's final callback, on that same thread."""

    @staticmethod
    def forward(ctx, x, rec):
        ctx.rec = rec
        return x.view_as(x)

    @staticmethod
    def backward(ctx, g):
        rec = ctx.rec
        rec.begin()
        torch.autograd.Variable._execution_engine.queue_callback(rec.end)
        return g, None


class SegmentedStep:
    """forward + backward of one static batch shape as HIP graphs: the forward (and loss)
    as one graph captured on the calling thread, the backward as segments cut where a DDP
    bucket completes, captured on autograd's device thread.

    ``capture(fwd)`` runs ``fwd()`` -> (loss, *outputs) under capture (its tensors must be
    static: inputs copied into buffers the caller owns), then ``loss.backward()``; returns
    (loss, *outputs) as graph-owned static tensors refreshed by every replay.  ``replay()``
    re-runs it, launching each bucket's all-reduce between the backward segments."""

    def __init__(self, device, pool=None, stream=None):
        """``stream``: capture on this stream -- pass the side stream the eager warm-up steps
        ran on: autograd runs a parameter's gradient accumulation on the stream its
        accumulator was created on, and a cut must not leave work forked onto another
        stream unjoined."""
        self.device = torch.device(device)
        self.pool = pool if pool is not None else torch.cuda.graph_pool_handle()
        self.stream = stream
        self.fwd = None
        self.rec = None
        self.one = None

    def capture(self, fwd):
        side = self.stream if self.stream is not None else torch.cuda.Stream(device=self.device)
        side.wait_stream(torch.cuda.current_stream(self.device))
        torch.cuda.synchronize(self.device)
        rec = Recorder(self.pool)
        from ..ops.mixup import unit_grad
        self.one = unit_grad(self.device)  # static seed gradient of the loss (the loss node skips its scaling)
        with torch.cuda.stream(side):
            # the forward is a Recorder too: FSDP's per-unit gathers (static mode) cut it into
            # segments, each unit's all-gather wait / next-unit prefetch between them
            frec = Recorder(self.pool)
            frec.stream = side
            with recording(frec), capture_guard():
                frec.begin()
                try:
                    out = fwd()
                    loss = _BackwardCaptureStart.apply(out[0], rec)
                finally:
                    frec.end()
            self.fwd = frec
            assert loss.dim() == 0 and loss.dtype == torch.float32, "SegmentedStep: scalar fp32 loss"
            with recording(rec), capture_guard():
                loss.backward(self.one)
        torch.cuda.current_stream(self.device).wait_stream(side)
        assert rec.cur is None and rec.segments, "backward capture did not complete"
        self.rec = rec
        return out

    @property
    def num_segments(self):
        return len(self.fwd.segments) + (len(self.rec.segments) if self.rec else 0)

    def replay(self):
        self.fwd.replay()
        self.rec.replay()


# ------------------------------------------------------------------ capture guard
class CaptureUnsafeOp(RuntimeError):
    pass


# ATen ops whose output size depends on tensor VALUES (or that read a device value back to
# the host): under HIP-graph capture they either synchronise (illegal while capturing) or,
# worse, size their buffers from a value read at capture time, so a replay with other data
# writes out of bounds (round-2: rocprim partition_kernel aperture violation on replay of
# the torch-op transformer step, from embedding_dense_backward's unique-by-key).
_UNSAFE = ("nonzero", "masked_select", "unique", "_unique", "unique_consecutive", "unique_dim",
           "_unique2", "embedding_dense_backward", "_local_scalar_dense", "repeat_interleave",
           "masked_scatter", "_embedding_bag_backward", "bincount", "histc")


def _on_device(args, kwargs):
    def dev(x):
        if isinstance(x, torch.Tensor):
            return x.device.type != "cpu"
        if isinstance(x, (list, tuple)):
            return any(dev(y) for y in x)
        return False
    return dev(args) or dev(list((kwargs or {}).values()))


class _CaptureGuardMode(TorchDispatchMode):
    def __torch_dispatch__(self, func, types, args=(), kwargs=None):
        name = func.overloadpacket.__name__
        if name in _UNSAFE and _on_device(args, kwargs):  # (host tensors are not captured)
            raise CaptureUnsafeOp(f"{func} inside a HIP-graph capture: its output size / host value depends on the "
                                  f"data, so replays would reuse the capture-time size (not graph-safe)")
        if name == "index" and _on_device(args, kwargs) and any(
                isinstance(t, torch.Tensor) and t.dtype == torch.bool for t in (args[1] if len(args) > 1 else ())):
            raise CaptureUnsafeOp("boolean-mask indexing inside a HIP-graph capture (data-dependent output size)")
        return func(*args, **(kwargs or {}))


@contextlib.contextmanager
def capture_guard():
    """Raise ``CaptureUnsafeOp`` when a data-dependent-size or host-synchronising ATen op runs
    inside the block (every HIP-graph capture of this package is wrapped in it; the mode is
    part of the thread-local state autograd hands to its device threads, so backward ops are
    checked too)."""
    with _CaptureGuardMode():
        yield
