#!/usr/bin/env python3
"""Does a main-stream kernel run while the batched Jacobi eigensolver runs on a side stream?

The transformer's NGD update step launches ``jacobi_eigh`` on a side stream (optim/ngd.py
``drive``) so that it overlaps the next training step; a kernel trace at 32 samples / GPU
showed the main stream idle for the whole ~1.4 ms of every eigensolve.  Times:
  [a] eigh alone, [b] main-stream sleep alone, [c] eigh on side + sleep on main launched
  right after, [d] the same with the host launching the sleep first.
"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from faster_distributed_training_amd.ops import eigh as E  # noqa: E402


def ev():
    return torch.cuda.Event(enable_timing=True)


def main():
    torch.cuda.init()
    dev = torch.device("cuda")
    g = torch.Generator(device="cpu").manual_seed(0)
    A = torch.randn(147, 80, 80, generator=g)
    Z = (A @ A.transpose(1, 2)).to(dev)
    side = torch.cuda.Stream()
    torch.cuda._sleep(1000)
    E.batched_eigh(Z)
    torch.cuda.synchronize()
    s, e = ev(), ev()
    s.record(); E.batched_eigh(Z); e.record(); torch.cuda.synchronize()
    t_eigh = s.elapsed_time(e)
    s.record(); torch.cuda._sleep(1 << 21); e.record(); torch.cuda.synchronize()
    t_sleep = s.elapsed_time(e)
    print(f"[a] eigh alone {t_eigh:.3f} ms   [b] sleep alone {t_sleep:.3f} ms", flush=True)
    with torch.cuda.stream(side):  # (the first launch on a stream creates its queue: ~5 ms)
        E.batched_eigh(Z)
    torch.cuda.synchronize()
    for order in ("eigh_first", "sleep_first"):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        s.record()
        side.wait_stream(torch.cuda.current_stream())
        if order == "eigh_first":
            with torch.cuda.stream(side):
                E.batched_eigh(Z)
            th = time.perf_counter()
            torch.cuda._sleep(1 << 21)
        else:
            torch.cuda._sleep(1 << 21)
            with torch.cuda.stream(side):
                E.batched_eigh(Z)
            th = time.perf_counter()
        torch.cuda.current_stream().wait_stream(side)
        e.record()
        host = (time.perf_counter() - t0) * 1e3
        torch.cuda.synchronize()
        tot = s.elapsed_time(e)
        verdict = "CONCURRENT" if tot < 0.8 * (t_eigh + t_sleep) else "SERIALISED"
        print(f"[{order}] both {tot:.3f} ms (sum {t_eigh + t_sleep:.3f}) -> {verdict}; host launch "
              f"{(th - t0) * 1e3:.3f} ms, host total {host:.3f} ms", flush=True)
    # the optimizer's pattern: main work, side waits on main, cat + eigh + small kernels on
    # side, then small main-stream kernels (foreach copy) + a sleep: when does main finish?
    xs = [torch.randn(512, 512, device=dev) for _ in range(40)]
    ys = [torch.empty_like(t) for t in xs]
    for _ in range(2):
        torch.cuda.synchronize()
        s.record()
        torch.cuda._sleep(1 << 18)
        side.wait_stream(torch.cuda.current_stream())
        e_side = ev()
        with torch.cuda.stream(side):
            Zc = torch.cat([Z.reshape(-1)]).view_as(Z)
            E.batched_eigh(Zc)
            for t in xs[:8]:
                t.mul_(1.0)
            e_side.record(side)
        torch._foreach_copy_(ys, xs)
        torch.cuda._sleep(1 << 20)
        e.record()
        torch.cuda.synchronize()
        print(f"[pattern] main done at {s.elapsed_time(e):.3f} ms, side done at {s.elapsed_time(e_side):.3f} ms "
              f"-> main {'OVERLAPPED the eigh' if s.elapsed_time(e) < s.elapsed_time(e_side) else 'waited'}", flush=True)
    # a GEMM stream on main against the eigh on side
    a = torch.randn(4096, 4096, device=dev, dtype=torch.bfloat16)
    for _ in range(3):
        a @ a
    torch.cuda.synchronize()
    s.record()
    for _ in range(20):
        a @ a
    e.record(); torch.cuda.synchronize()
    t_mm = s.elapsed_time(e)
    s.record()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        E.batched_eigh(Z)
    for _ in range(20):
        a @ a
    torch.cuda.current_stream().wait_stream(side)
    e.record(); torch.cuda.synchronize()
    print(f"[gemm] 20 GEMMs alone {t_mm:.3f} ms, with the side eigh {s.elapsed_time(e):.3f} ms", flush=True)


def trainer_host_times(steps=24):
    """Host time of the side-stream calls inside the real transformer NGD step (32 samples)."""
    import faster_distributed_training_amd.ops.eigh as Emod
    from faster_distributed_training_amd.optim import ngd as ngd_mod
    from faster_distributed_training_amd.train.transformer_trainer import TransformerConfig, TransformerTrainer
    acc = {"eigh_many": [], "post_update": [], "drive": [], "foreach_copy": []}

    def timed(name, fn):
        def w(*a, **k):
            t = time.perf_counter()
            r = fn(*a, **k)
            acc[name].append((time.perf_counter() - t) * 1e3)
            return r
        return w
    Emod.eigh_many = timed("eigh_many", Emod.eigh_many)
    ngd_mod.NGState._post_update = timed("post_update", ngd_mod.NGState._post_update)
    ngd_mod.drive = timed("drive", ngd_mod.drive)
    torch._foreach_copy_ = timed("foreach_copy", torch._foreach_copy_)
    tr = TransformerTrainer(TransformerConfig(batch_size=32, synthetic=True, eval=False, plot=False, ngd=True,
                                              length_buckets=(128, 256), epoch=1))
    it = iter(tr.train_loader)
    tr.model.train()
    for _ in range(15):
        tr.train_step(*next(it))
    torch.cuda.synchronize()
    for v in acc.values():
        v.clear()
    t0 = time.perf_counter()
    for _ in range(steps):
        tr.train_step(*next(it))
    host = (time.perf_counter() - t0) / steps * 1e3
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / steps * 1e3
    print(f"[trainer] host {host:.3f} ms / step, wall {wall:.3f} ms / step", flush=True)
    for k, v in acc.items():
        if v:
            print(f"   {k:13s} calls {len(v):4d}  mean {sum(v) / len(v):.3f} ms  max {max(v):.3f} ms  "
                  f"total/step {sum(v) / steps:.3f} ms", flush=True)


if __name__ == "__main__":
    main()
    trainer_host_times()
