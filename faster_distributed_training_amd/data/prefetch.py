"""Pinned-host -> device batch staging on a dedicated copy stream (survey D4/D7).

Reference: ``DataLoaderX`` (prefetch_generator.BackgroundGenerator) + ``pin_memory=True``
+ ``.to(device, non_blocking=True)`` (resnet50_test.py:41-43,321-340,522;
transformer_test.py:68-70,106-138,242-245).

MI355X design: the native ``PinnedPrefetcher`` (csrc/runtime/runtime.cpp) owns a ring of
pinned host slots (hipHostMalloc) and a non-blocking HIP copy stream; ``stage_many``
memcpy's a host batch into a free pinned slot with the GIL released and enqueues the
``hipMemcpyAsync`` H2D on the copy stream.  This module adds the device half of the ring:

* one device buffer per slot, so a staged batch is never overwritten while the compute
  stream still reads it: before the copy into slot ``s`` the copy stream waits on the
  event the compute stream recorded when it enqueued the last reader of ``s``
  (``release``);
* ``acquire(s)`` makes the compute stream wait on the copy's event (hipStreamWaitEvent):
  no host blocking, the H2D of batch k+1 overlaps the step of batch k.

Loaders stage batch k+1 before handing out batch k (``StagedIterator``), so with 3 slots
the copy of the next batch, the step on the current one and the host gather of the one
after overlap.  Nothing here ever does a pageable ``.to(device)``.
"""
from __future__ import annotations

import numpy as np
import torch

from ..ops import _native

_ALIGN = 256


def _aligned(n: int) -> int:
    return (n + _ALIGN - 1) // _ALIGN * _ALIGN


class PinnedStager:
    """Ring of (pinned host slot, device slot, copy event, release event)."""

    def __init__(self, device, slot_bytes: int, nslots: int = 3):
        assert nslots >= 3, "one slot in copy, one in use, one free"
        self.device = torch.device(device)
        nat = _native.native()
        self.slot_bytes = _aligned(int(slot_bytes))
        self.pf = nat.PinnedPrefetcher(self.device.index or 0, self.slot_bytes, nslots)
        self.nslots = nslots
        self.dev = [torch.empty(self.slot_bytes, dtype=torch.uint8, device=self.device) for _ in range(nslots)]
        self.released: list[torch.cuda.Event | None] = [None] * nslots
        self.copy_stream = torch.cuda.ExternalStream(self.pf.copy_stream, device=self.device)
        # the device slots come from the compute stream's allocator pool: the first copies
        # must not overtake compute work still pending on that memory
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(self.device))
        self.copy_stream.wait_event(ev)
        self.next = 0
        self.staged = 0  # batches staged (tests / diagnostics)

    def stage(self, arrays):
        """Copy host arrays (numpy or CPU tensors) to the device through the next slot.
        Returns (slot, [device tensors with the arrays' dtypes and shapes]); the tensors
        may be read on the compute stream only after ``acquire(slot)``."""
        s = self.next
        self.next = (s + 1) % self.nslots
        ev = self.released[s]
        if ev is not None:
            self.copy_stream.wait_event(ev)  # the slot's previous readers are done
        srcs, sizes, dsts, outs, keep = [], [], [], [], []
        off = 0
        for a in arrays:
            t = torch.from_numpy(np.ascontiguousarray(a)) if isinstance(a, np.ndarray) else a.contiguous()
            assert t.device.type == "cpu"
            n = t.numel() * t.element_size()
            if off + n > self.slot_bytes:
                raise ValueError(f"batch of {off + n} B exceeds the {self.slot_bytes} B staging slot")
            keep.append(t)
            srcs.append(t.data_ptr())
            sizes.append(n)
            dsts.append(self.dev[s].data_ptr() + off)
            outs.append(self.dev[s][off:off + n].view(t.dtype).view(t.shape))
            off += _aligned(n)
        got = self.pf.stage_many(srcs, sizes, dsts)  # memcpy to pinned (GIL released) + async H2D
        assert got == s, (got, s)
        self.staged += 1
        return s, outs

    def acquire(self, s: int):
        """Order the current compute stream after slot ``s``'s H2D copy (device-side wait)."""
        self.pf.wait(s, _native.stream_ptr(self.device))

    def release(self, s: int):
        """Every compute-stream reader of slot ``s`` has been enqueued: the next copy into
        the slot waits for them."""
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(self.device))
        self.released[s] = ev

    def synchronize(self):
        self.pf.synchronize()


class StagedIterator:
    """Runs ``host(b) -> (arrays, meta)`` + ``stage`` one batch ahead of
    ``device(arrays, meta) -> batch``.

    ``host`` builds batch b's host arrays (gather/pad in numpy) plus host-side metadata
    (e.g. the padded length); ``device`` turns the staged device tensors into the batch
    the trainer consumes (gathers, casts, GPU augmentation) on the compute stream."""

    def __init__(self, stager: PinnedStager, nb: int, host, device):
        self.stager, self.nb, self.host, self.device = stager, nb, host, device

    def _stage(self, b):
        arrays, meta = self.host(b)
        return self.stager.stage(arrays), meta

    def __iter__(self):
        st = self.stager
        pending = self._stage(0) if self.nb > 0 else None
        for b in range(self.nb):
            nxt = self._stage(b + 1) if b + 1 < self.nb else None  # in flight during step b
            (s, arrs), meta = pending
            st.acquire(s)
            out = self.device(arrs, meta)
            st.release(s)
            yield out
            pending = nxt
