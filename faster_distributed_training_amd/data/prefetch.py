"""Pinned-host -> device batch staging on a dedicated copy stream (survey D4/D7).

Reference: ``DataLoaderX`` (prefetch_generator.BackgroundGenerator) + ``pin_memory=True``
+ ``.to(device, non_blocking=True)`` (resnet50_test.py:41-43,321-340,522;
transformer_test.py:68-70,106-138,242-245).

MI355X design: the native ``PinnedPrefetcher`` (csrc/runtime/runtime.cpp) owns a ring of
pinned host slots (hipHostMalloc), a non-blocking HIP copy stream and a C++ worker thread;
``submit`` queues a host batch to the worker, which waits for the slot's previous H2D,
memcpy's the batch into the pinned slot and enqueues the ``hipMemcpyAsync`` on the copy
stream -- the training thread never does the copy (the reference's pin-memory thread).
The host half of a batch (the numpy gather) runs ahead in a Python background thread
(``StagedIterator``, the reference's ``BackgroundGenerator``).  This module adds the device
half of the ring:

* one device buffer per slot, so a staged batch is never overwritten while the compute
  stream still reads it: before the copy into slot ``s`` the copy stream waits on the
  event the compute stream recorded when it enqueued the last reader of ``s``
  (``release``);
* ``acquire(s)`` makes the compute stream wait on the copy's event (hipStreamWaitEvent):
  no host blocking, the H2D of batch k+1 overlaps the step of batch k.

Loaders stage batch k+1 before handing out batch k (``StagedIterator``), so with 3 slots
the copy of the next batch, the step on the current one and the host gather of the one
after (background thread) overlap.  Nothing here ever does a pageable ``.to(device)``.
"""
from __future__ import annotations

import queue
import threading
import time

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
        # host seconds spent blocked in acquire(): the ring's backpressure (the worker waits for
        # the GPU to release a slot before it can issue the next copy) -- time the training
        # thread is idle because the GPU is behind, not host work (bench.py host_busy_ms_per_step)
        self.wait_s = 0.0
        self._keep: list = [None] * nslots  # sources + release event alive until the job is issued

    def stage(self, arrays):
        """Copy host arrays (numpy or CPU tensors) to the device through the next slot.
        Returns (slot, [device tensors with the arrays' dtypes and shapes]); the tensors
        may be read on the compute stream only after ``acquire(slot)``.  The copy itself is
        done by the native worker thread (``PinnedPrefetcher.submit``); the copy stream first
        waits for the slot's previous readers (their release event)."""
        s = self.next
        self.next = (s + 1) % self.nslots
        if self._keep[s] is not None:
            # the slot's previous job was never acquired (abandoned iterator): its sources
            # must outlive the worker's memcpy from them before they are replaced below
            self.pf.wait_issued(s)
        ev = self.released[s]
        srcs, sizes, dsts, outs, keep = [], [], [], [], [ev]
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
        got = self.pf.submit(srcs, sizes, dsts, ev.cuda_event if ev is not None else 0)
        assert got == s, (got, s)
        self._keep[s] = keep
        self.staged += 1
        return s, outs

    def acquire(self, s: int):
        """Order the current compute stream after slot ``s``'s H2D copy (device-side wait; the
        host only waits for the worker to have ISSUED the copy)."""
        t0 = time.perf_counter()
        self.pf.wait(s, _native.stream_ptr(self.device))
        self.wait_s += time.perf_counter() - t0
        self._keep[s] = None

    def release(self, s: int):
        """Every compute-stream reader of slot ``s`` has been enqueued: the next copy into
        the slot waits for them."""
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(self.device))
        self.released[s] = ev

    def synchronize(self):
        self.pf.synchronize()


class _Producer:
    """Background host producer (the reference's ``prefetch_generator.BackgroundGenerator``):
    a daemon thread computes ``host(b)`` for b = 0..nb-1 in order into a bounded queue
    (``depth`` batches ahead); numpy's gathers release the GIL, so they overlap the training
    thread's kernel launches.  Exceptions are re-raised in the consumer."""

    _END = object()

    def __init__(self, host, nb: int, depth: int = 2):
        self.q: queue.Queue = queue.Queue(maxsize=depth)
        self.stop = threading.Event()
        self.t = threading.Thread(target=self._run, args=(host, nb), daemon=True, name="fdt-host-producer")
        self.t.start()

    def _put(self, x) -> bool:
        while not self.stop.is_set():
            try:
                self.q.put(x, timeout=0.1)
                return True
            except queue.Full:
                continue
        return False

    def _run(self, host, nb):
        try:
            for b in range(nb):
                if not self._put((None, host(b))):
                    return
            self._put((None, self._END))
        except BaseException as e:  # noqa: BLE001 -- handed to the consumer
            self._put((e, None))

    def get(self):
        err, item = self.q.get()
        if err is not None:
            raise err
        return item

    def close(self):
        self.stop.set()
        try:
            while True:
                self.q.get_nowait()
        except queue.Empty:
            pass
        self.t.join(timeout=5)


class StagedIterator:
    """Runs ``host(b) -> (arrays, meta)`` in a background thread and ``stage`` one batch ahead
    of ``device(arrays, meta) -> batch``.

    ``host`` builds batch b's host arrays (gather/pad in numpy) plus host-side metadata
    (e.g. the padded length) -- it must be a pure function of b (it runs on another thread);
    ``device`` turns the staged device tensors into the batch the trainer consumes (gathers,
    casts, GPU augmentation) on the compute stream.  ``background=False``: host(b) inline."""

    def __init__(self, stager: PinnedStager, nb: int, host, device, background: bool = True, depth: int = 2):
        self.stager, self.nb, self.host, self.device = stager, nb, host, device
        self.background, self.depth = background, depth

    def __iter__(self):
        st = self.stager
        prod = _Producer(self.host, self.nb, self.depth) if (self.background and self.nb > 1) else None

        def stage(b):
            arrays, meta = prod.get() if prod is not None else self.host(b)
            return st.stage(arrays), meta

        try:
            pending = stage(0) if self.nb > 0 else None
            for b in range(self.nb):
                nxt = stage(b + 1) if b + 1 < self.nb else None  # in flight during step b
                (s, arrs), meta = pending
                st.acquire(s)
                out = self.device(arrs, meta)
                st.release(s)
                yield out
                pending = nxt
        finally:
            if prod is not None:
                prod.close()
