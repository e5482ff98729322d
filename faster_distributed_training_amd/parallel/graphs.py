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
transformer trainer under DDP).  Reference: DDP's bucketed overlap
(``resnet50_test.py:716``, ``transformer_test.py:241-271``).
"""
from __future__ import annotations

import torch

# The recorder of the capture in progress (read by parallel/ddp.py hooks and the engine's
# grad_ready from the autograd thread); None outside a capture.
_ACTIVE = None


def active():
    return _ACTIVE


class Recorder:
    """Capture split into graph segments at deferred hook actions.

    ``mode``: the stream-capture mode.  "thread_local" when every begin / cut / end happens
    on one thread (the engine's backward); "global" when the capture starts on the main
    thread and is cut from autograd's device thread (``SegmentedStep``).  A cut always
    ends and restarts the capture on the stream it began on, after joining the caller's
    current stream if autograd runs the hook on another (forked, captured) stream."""

    def __init__(self, pool, mode="thread_local"):
        self.pool = pool
        self.mode = mode
        self.segments = []  # [(CUDAGraph, [actions to run after it])]
        self.cur = None
        self.stream = None
        self.foreign_cuts = 0  # cuts requested from a stream other than the capture stream

    def begin(self):
        if self.stream is None:
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
        with torch.cuda.stream(self.stream):
            self.cur.capture_end()
        self.segments.append((self.cur, list(actions)))
        self.begin()

    def end(self):
        self._join()
        with torch.cuda.stream(self.stream):
            self.cur.capture_end()
        self.segments.append((self.cur, []))
        self.cur = None

    def replay(self):
        for graph, acts in self.segments:
            graph.replay()
            for a in acts:
                a()


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


class SegmentedStep:
    """forward + backward of one static batch shape as segmented HIP graphs.

    ``capture(fn)`` runs ``fn()`` (forward, loss, ``loss.backward()``; its tensors must be
    static: inputs copied into buffers the caller owns) under capture on a side stream and
    returns fn's outputs (graph-owned static tensors, refreshed by every replay);
    ``replay()`` re-runs it, launching the bucket all-reduces between segments."""

    def __init__(self, device, pool=None):
        self.device = torch.device(device)
        self.pool = pool if pool is not None else torch.cuda.graph_pool_handle()
        self.rec = None

    def capture(self, fn):
        side = torch.cuda.Stream(device=self.device)
        side.wait_stream(torch.cuda.current_stream(self.device))
        torch.cuda.synchronize(self.device)
        rec = Recorder(self.pool, mode="global")
        with torch.cuda.stream(side), recording(rec):
            rec.begin()
            try:
                out = fn()
            finally:
                rec.end()
        torch.cuda.current_stream(self.device).wait_stream(side)
        self.rec = rec
        return out

    @property
    def num_segments(self):
        return len(self.rec.segments) if self.rec else 0

    def replay(self):
        self.rec.replay()
