"""Process-group bootstrap / teardown and the metric all-reduce.

Reference: ``utils.py:13-34`` (``setup``, ``setup_norank``, ``setup_sharedfile``,
``cleanup``), ``resnet50_test.py:616-619`` (metric all-reduce, X7).

MI355X design: one process per GPU, ``torch.distributed`` with backend ``nccl`` (which
IS RCCL on ROCm) over xGMI; ``gloo`` for CPU runs and tests.  The device is
``LOCAL_RANK`` (the reference used the global rank — single-node only, survey Q15).
``HSA_ENABLE_IPC_MODE_LEGACY=0`` is kept in the environment (dmabuf IPC; required by
RCCL on this platform).
"""
from __future__ import annotations

import datetime
import os

import torch
import torch.distributed as dist

from ..utils.env import env_int, local_rank


def _backend():
    """``nccl`` (= RCCL) on GPUs, ``gloo`` on CPU; ``FDT_DIST_BACKEND`` overrides (e.g. gloo
    to rehearse several ranks on one GPU, which RCCL does not allow)."""
    be = os.environ.get("FDT_DIST_BACKEND")
    if be:
        return be
    return "nccl" if torch.cuda.is_available() else "gloo"


def _comm_env():
    """RCCL's collective streams come from the high-priority pool.  Measured (round 3, a
    kernel trace of the DDP path at world 1): from the normal pool the stream
    ProcessGroupNCCL took landed on the SAME hardware queue as the compute stream (HIP shares
    GPU_MAX_HW_QUEUES = 4 queues round-robin), so every bucket all-reduce executed in queue
    order between two backward kernels and could never overlap them; high-priority streams
    get their own queue (``profiles/r3s3/ddp_queues.txt``)."""
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    os.environ.setdefault("TORCH_NCCL_HIGH_PRIORITY", "1")
    # No recycled collective events: the bucket all-reduces captured into the backward graph
    # record their completion events inside the capture, and torch's event cache hands such an
    # event to a later eager collective; once (closing run of round 5, the capture-check
    # fallback test) RCCL's watchdog thread then failed querying "an event last recorded in a
    # capturing stream" and aborted the process.  A fresh event per eager collective costs
    # microseconds (in capture mode the step's collectives are graph nodes).
    os.environ.setdefault("TORCH_NCCL_CUDA_EVENT_CACHE", "0")


def _bind_device():
    if torch.cuda.is_available():
        torch.cuda.set_device(local_rank() % torch.cuda.device_count())


def setup(rank: int = 0, world_size: int = 1, master_addr: str = "127.0.0.1", master_port: int = 12355,
          backend: str | None = None, timeout_s: int = 1800):
    """Explicit-rank bootstrap (reference ``setup``, ``utils.py:13-17``)."""
    _comm_env()
    os.environ.setdefault("MASTER_ADDR", master_addr)
    os.environ.setdefault("MASTER_PORT", str(master_port))
    os.environ.setdefault("LOCAL_RANK", str(rank))
    _bind_device()
    be = backend or _backend()
    kw = dict(rank=rank, world_size=world_size, timeout=datetime.timedelta(seconds=timeout_s))
    if be == "nccl" and torch.cuda.is_available():
        kw["device_id"] = torch.device("cuda", torch.cuda.current_device())
    dist.init_process_group(be, **kw)
    return dist.get_rank(), dist.get_world_size()


def setup_norank(world_size: int | None = None, backend: str | None = None, timeout_s: int = 1800):
    """torchrun bootstrap: rank/world from the environment (reference ``setup_norank``,
    ``utils.py:20-23`` — the path the reference actually uses)."""
    _comm_env()
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "12355")
    _bind_device()
    be = backend or _backend()
    kw = dict(timeout=datetime.timedelta(seconds=timeout_s))
    if be == "nccl" and torch.cuda.is_available():
        kw["device_id"] = torch.device("cuda", torch.cuda.current_device())
    if "RANK" not in os.environ:
        kw.update(rank=0, world_size=world_size or 1)
    dist.init_process_group(be, **kw)
    return dist.get_rank(), dist.get_world_size()


def setup_sharedfile(world_size: int, path: str = "/tmp/fdt_sharedfile", backend: str | None = None,
                     rank: int | None = None):
    """File-store rendezvous for multi-node on a shared filesystem (reference
    ``setup_sharedfile``, ``utils.py:26-30``)."""
    _comm_env()
    _bind_device()
    r = rank if rank is not None else env_int("RANK", 0)
    dist.init_process_group(backend or _backend(), init_method=f"file://{path}", world_size=world_size, rank=r)
    return dist.get_rank(), dist.get_world_size()


def cleanup():
    if dist.is_initialized():
        dist.destroy_process_group()


def is_dist():
    return dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1


def rank():
    return dist.get_rank() if dist.is_initialized() else 0


def world():
    return dist.get_world_size() if dist.is_initialized() else 1


def barrier():
    if dist.is_initialized():
        if dist.get_backend() == "nccl":
            dist.barrier(device_ids=[torch.cuda.current_device()])
        else:
            dist.barrier()


@torch.no_grad()
def broadcast_buffers(module, src: int = 0, group=None):
    """Broadcast the floating-point buffers of ``module`` (BatchNorm running statistics)
    from ``src`` in ONE collective (DDP ``broadcast_buffers``, X3)."""
    if module is None or not is_dist():
        return
    bufs = [b for b in module.buffers() if b.dtype.is_floating_point]
    if not bufs:
        return
    flat = torch.cat([b.reshape(-1) for b in bufs])
    dist.broadcast(flat, src, group=group)
    off = 0
    for b in bufs:
        n = b.numel()
        b.copy_(flat[off:off + n].view_as(b))
        off += n


def broadcast_scalar(value: float, src: int = 0, device=None) -> float:
    """``value`` as seen by rank ``src`` (collective decisions such as "save a new best
    checkpoint" must be taken identically on every rank)."""
    if not is_dist():
        return float(value)
    if device is None:
        device = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend() == "nccl" else "cpu"
    t = torch.tensor([float(value)], dtype=torch.float64, device=device)
    dist.broadcast(t, src)
    return float(t.item())


def all_reduce_metrics(*tensors: torch.Tensor, op=dist.ReduceOp.SUM):
    """Metric all-reduce (X7): one collective for all metric scalars (the reference
    issues one per scalar).  Tensors are reduced in place."""
    if not is_dist() or not tensors:
        return tensors
    flat = torch.cat([t.reshape(-1).float() for t in tensors])
    dist.all_reduce(flat, op=op)
    off = 0
    for t in tensors:
        n = t.numel()
        t.copy_(flat[off:off + n].view_as(t).to(t.dtype))
        off += n
    return tensors


def average_gradients(model, world_size: int | None = None):
    """Manual gradient averaging (reference ``average_gradients``,
    ``resnet50_test.py:499-502``, which hard-codes /4): one all-reduce per parameter.
    Kept for API parity; the trainer uses ``parallel.ddp.BucketReducer``."""
    ws = world_size or world()
    for p in model.parameters():
        if p.grad is not None:
            dist.all_reduce(p.grad, op=dist.ReduceOp.SUM)
            p.grad.div_(ws)


def distributed_wrapper(rank_, world_size, func, *func_args, backend=None, port=12355):
    """``mp.spawn`` target (reference ``distributed_wrapper``, ``utils.py:37-46``; the
    reference's argument order is broken, survey P3 — this one matches mp.spawn's
    ``(rank, *args)`` contract)."""
    os.environ["LOCAL_RANK"] = str(rank_)
    setup(rank_, world_size, master_port=port, backend=backend)
    try:
        return func(rank_, world_size, *func_args)
    finally:
        cleanup()


def distributed_wrapper_runner(func, world_size, *func_args, backend=None, port=12355):
    """Spawn ``world_size`` processes running ``func(rank, world_size, *args)``."""
    import torch.multiprocessing as mp
    mp.spawn(_spawn_entry, args=(world_size, func, func_args, backend, port), nprocs=world_size, join=True)


def _spawn_entry(rank_, world_size, func, func_args, backend, port):
    distributed_wrapper(rank_, world_size, func, *func_args, backend=backend, port=port)


distributed_warpper_runner = distributed_wrapper_runner  # reference spelling (utils.py:49)
