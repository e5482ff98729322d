"""Multi-process harness for distributed tests on the CPU (gloo backend, 127.0.0.1)."""
from __future__ import annotations

import os
import socket
import sys
import traceback

import torch.multiprocessing as mp


def free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _entry(rank, world, port, fn, args, errq, native=False, backend="gloo"):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    os.environ["RANK"] = str(rank)
    os.environ["LOCAL_RANK"] = str(rank)
    os.environ["WORLD_SIZE"] = str(world)
    os.environ["FDT_NATIVE"] = "1" if native else "0"
    try:
        import torch.distributed as dist
        if backend == "nccl":  # RCCL: one process per device; bind it before the group exists
            import torch
            from faster_distributed_training_amd.parallel.dist import _comm_env
            _comm_env()  # (the package's RCCL environment defaults)
            torch.cuda.set_device(rank)
            dist.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device("cuda", rank))
        else:
            dist.init_process_group("gloo", rank=rank, world_size=world)
        try:
            fn(rank, world, *args)
            # gloo tears down its pair threads in destroy_process_group; a rank that leaves while
            # its peer still has a send in flight can abort the peer (std::terminate) under load
            dist.barrier()
        finally:
            dist.destroy_process_group()
    except Exception:  # report to the parent
        errq.put((rank, traceback.format_exc()))
        sys.exit(1)


def run_world(fn, world=2, args=(), timeout=240, native=False, backend="gloo"):
    """Spawn ``world`` ranks (gloo).  native=True keeps the HIP fast path on (GPU tests:
    every rank shares cuda:0 -- gloo, unlike RCCL, allows several ranks per device);
    backend="nccl" runs RCCL (one rank per GPU: world 1 on the single-GPU test box)."""
    ctx = mp.get_context("spawn")
    errq = ctx.SimpleQueue()
    port = free_port()
    procs = [ctx.Process(target=_entry, args=(r, world, port, fn, args, errq, native, backend))
             for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout)
    for p in procs:
        if p.is_alive():
            p.kill()
            raise RuntimeError("distributed test timed out")
    errs = []
    while not errq.empty():
        errs.append(errq.get())
    if errs or any(p.exitcode != 0 for p in procs):
        raise AssertionError("\n".join(f"rank {r}:\n{tb}" for r, tb in errs) or "a rank failed")
