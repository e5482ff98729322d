"""One rank of a world-N data-parallel job, rehearsed on ONE GPU (``bench.py --simulate-world N
--simulate-rank R``).

The 8-GPU runs belong to the driver, yet the per-rank step of the 8-GPU configurations --
batch 1024/N per rank, rank R's 1/N owner shard of the NGD state (``parallel/zero.py``), rank
R's FSDP shards (``parallel/fsdp.py``), the DDP bucket plan and the in-graph collectives of
``parallel/graphs.py`` -- is fully determined by (R, N).  ``install(R, N)`` makes this process
BE rank R of a world-N ``nccl`` job as far as the framework can tell, with every collective
replaced by a same-sized local operation on the device:

* ``all_reduce(t)``: SUM -> ``t *= N`` (the magnitude an all-reduce of N similar contributions
  has), AVG / MAX / MIN -> ``t *= 1`` -- one read + one write of the buffer in place, the HBM
  traffic of RCCL's reduction kernels on this rank;
* ``reduce_scatter_tensor(out, inp)``: out = inp[R-th slice] (x N for SUM), plus one in-place
  read + write of ``inp``;
* ``all_gather_into_tensor(out, inp)``: out[R-th slice] = inp (the other slices keep this rank's
  replica of those parameters, which every rank initialised identically), plus one in-place
  read + write of ``out``;
(no scratch buffers: a collective captured into a HIP graph must not allocate from the capture's
private pool and keep the block past it)
* ``broadcast`` / ``barrier``: no-ops (rank-0 values are this rank's own).

``async_op=True`` collectives run on a side stream forked from the current one and joined by
``Work.wait()`` -- the overlap RCCL's own stream gives -- so they also capture into HIP graphs.
What this does NOT time is the xGMI transfer itself: that is bytes / link bandwidth, reported
separately (``comm_bytes``) for the reader to add under the overlap the trace shows.
"""
from __future__ import annotations

import torch
import torch.distributed as dist

_STATE = None


class _Work:
    def __init__(self, ev):
        self.ev = ev

    def wait(self):
        if self.ev is not None:
            torch.cuda.current_stream().wait_event(self.ev)
        return True

    def is_completed(self):
        return True


class _Sim:
    def __init__(self, rank: int, world: int):
        assert 0 <= rank < world, (rank, world)
        self.rank, self.world = rank, world
        self.side = None
        self.bytes = {"all_reduce": 0, "reduce_scatter": 0, "all_gather": 0}
        self.saved = {}

    def _run(self, fn, t: torch.Tensor, async_op: bool):
        if not (async_op and t.is_cuda):
            fn()
            return _Work(None) if async_op else None
        if self.side is None:
            self.side = torch.cuda.Stream(device=t.device)
        cur = torch.cuda.current_stream()
        self.side.wait_stream(cur)
        with torch.cuda.stream(self.side):
            fn()
            ev = torch.cuda.Event()
            ev.record(self.side)
        return _Work(ev)

    # -- collectives
    def all_reduce(self, t, op=dist.ReduceOp.SUM, group=None, async_op=False):
        self.bytes["all_reduce"] += t.numel() * t.element_size()

        def fn():
            t.mul_(self.world if op == dist.ReduceOp.SUM else 1)
        return self._run(fn, t, async_op)

    def reduce_scatter_tensor(self, out, inp, op=dist.ReduceOp.SUM, group=None, async_op=False):
        self.bytes["reduce_scatter"] += inp.numel() * inp.element_size()

        def fn():
            inp.mul_(1)
            out.copy_(inp.view(self.world, -1)[self.rank].view(out.shape))
            if op == dist.ReduceOp.SUM:
                out.mul_(self.world)
        return self._run(fn, out, async_op)

    def all_gather_into_tensor(self, out, inp, group=None, async_op=False):
        self.bytes["all_gather"] += out.numel() * out.element_size()

        def fn():
            out.mul_(1)
            out.view(self.world, -1)[self.rank].copy_(inp.reshape(-1))
        return self._run(fn, out, async_op)

    def broadcast(self, t, src=0, group=None, async_op=False):
        return _Work(None) if async_op else None

    def barrier(self, group=None, async_op=False, device_ids=None):
        return _Work(None) if async_op else None


def install(rank: int, world: int) -> None:
    """Make this process rank ``rank`` of a simulated world-``world`` nccl job (see module doc)."""
    global _STATE
    assert _STATE is None, "simulation already installed"
    s = _Sim(rank, world)
    backend = "nccl" if torch.cuda.is_available() else "gloo"  # the backend a real run of this box picks
    patches = {
        "is_available": lambda: True,
        "is_initialized": lambda: True,
        "get_rank": lambda group=None: s.rank,
        "get_world_size": lambda group=None: s.world,
        "get_backend": lambda group=None: backend,
        "init_process_group": lambda *a, **k: None,
        "destroy_process_group": lambda *a, **k: None,
        "all_reduce": s.all_reduce,
        "reduce_scatter_tensor": s.reduce_scatter_tensor,
        "all_gather_into_tensor": s.all_gather_into_tensor,
        "broadcast": s.broadcast,
        "barrier": s.barrier,
    }
    for k, v in patches.items():
        s.saved[k] = getattr(dist, k)
        setattr(dist, k, v)
    _STATE = s


def uninstall() -> None:
    global _STATE
    if _STATE is None:
        return
    for k, v in _STATE.saved.items():
        setattr(dist, k, v)
    _STATE = None


def active():
    return _STATE


def comm_bytes() -> dict:
    """Bytes this rank handed to each collective kind so far (0s when not simulating)."""
    return dict(_STATE.bytes) if _STATE is not None else {}
