#!/usr/bin/env python3
"""NGD optimizer step time on the real parameter sets (ResNet-50 CIFAR / Transformer 6x512),
random gradients, steady state (update and non-update steps of the schedule separately).

    python scripts/bench_ngd.py [--model resnet50|transformer] [--steps 24]
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="resnet50")
    ap.add_argument("--steps", type=int, default=24)
    ap.add_argument("--world", type=int, default=1,
                    help="simulate the ZeRO-2 sharded NGD of this many ranks: time each rank's shard optimizer")
    ap.add_argument("--balance", default="ngd", choices=["ngd", "numel"])
    ap.add_argument("--graphs", action="store_true", help="steady-state steps replayed as HIP graphs (NGD.graphs)")
    ap.add_argument("--gemm-micro", action="store_true",
                    help="time the update step's R x R products (ngd_gram / ngd_wupdate vs batched library GEMMs) "
                         "on every (G, R, D) preconditioner shape of the model")
    a = ap.parse_args()
    from faster_distributed_training_amd.optim.ngd import NGD
    from faster_distributed_training_amd.utils.flat import FlatParams
    dev = torch.device("cuda")
    if a.model == "resnet50":
        from faster_distributed_training_amd.models.resnet import resnet50
        m = resnet50(10)
    else:
        from faster_distributed_training_amd.models.transformer import Transformer
        m = Transformer(4, 30522)
    m = m.to(dev)
    if a.world > 1:
        from faster_distributed_training_amd.parallel.zero import ShardView
        full = FlatParams(m, device=dev, partition=a.world, balance=a.balance)
        per = []
        for r, (lo_s, hi_s) in enumerate(full.runs):
            v = ShardView(full, r * full.chunk, (r + 1) * full.chunk, full.slots[lo_s:hi_s])
            o = NGD(v, lr=0.01, momentum=0.9, weight_decay=1e-4)
            o.graphs = a.graphs
            per.append((r, time_steps(o, v, a.steps, dev)))
        for r, t in per:
            print(f"{a.model}: world {a.world} rank {r}: " + ", ".join(f"{k} median {v:.2f} ms" for k, v in t.items()))
        worst = {k: max(t[k] for _, t in per) for k in per[0][1]}
        print(f"{a.model}: world {a.world} ({a.balance}-balanced{', graphs' if a.graphs else ''}) slowest rank: " + ", ".join(f"{k} {v:.2f} ms" for k, v in worst.items()))
        return
    f = FlatParams(m, device=dev)
    o = NGD(f, lr=0.01, momentum=0.9, weight_decay=1e-4)
    o.graphs = a.graphs
    if a.gemm_micro:
        return gemm_micro(o, f, dev)
    g = torch.Generator(device=dev).manual_seed(0)
    times = {True: [], False: []}
    for s in range(a.steps):
        f.grad.normal_(generator=g)
        sts = o._states()
        upd = bool(sts) and sts[0]._updating()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        o.step()
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) * 1e3
        if s >= 2:
            times[upd].append(dt)
    n_axes = len(o._states())
    for k, v in times.items():
        if v:
            v.sort()
            print(f"{a.model}: {'update' if k else 'non-update'} steps: median {v[len(v) // 2]:.2f} ms "
                  f"(min {v[0]:.2f}, n={len(v)}), {n_axes} batched axis states")


def gemm_micro(o, f, dev):
    import faster_distributed_training_amd.optim.ngd as N
    f.grad.normal_()
    o.step()
    shapes = sorted({(st.G, st.rank, st.dim) for st in o._states() if st.rank > 0})

    def tm(fn, reps=20):
        for _ in range(3):
            fn()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        s.record()
        for _ in range(reps):
            fn()
        e.record()
        torch.cuda.synchronize()
        return s.elapsed_time(e) / reps * 1e3

    tot = {"gram": 0.0, "gram_lib": 0.0, "wupd": 0.0, "wupd_lib": 0.0}
    for G, R, D in shapes:
        J = torch.randn(G, R, D, device=dev)
        W = torch.randn(G, R, D, device=dev)
        A = torch.randn(G, R, R, device=dev)
        wc = torch.rand(G, R, device=dev)
        t = {}
        N.SMALL_GEMM = True
        t["gram"] = tm(lambda: N.gram(J, W))
        t["wupd"] = tm(lambda: N.w_update(A, J, wc, W))
        N.SMALL_GEMM = False
        t["gram_lib"] = tm(lambda: N.gram(J, W))
        t["wupd_lib"] = tm(lambda: N.w_update(A, J, wc, W))
        N.SMALL_GEMM = True
        for k in tot:
            tot[k] += t[k]
        print(f"G {G:3d} R {R:3d} D {D:5d}: gram {t['gram']:6.1f} us (lib {t['gram_lib']:6.1f})  "
              f"w-update {t['wupd']:6.1f} us (lib {t['wupd_lib']:6.1f})", flush=True)
    print("totals over the shapes (us): " + ", ".join(f"{k} {v:.1f}" for k, v in tot.items()))


def time_steps(o, f, steps, dev):
    g = torch.Generator(device=dev).manual_seed(0)
    times = {True: [], False: []}
    for s in range(steps):
        f.grad.normal_(generator=g)
        sts = o._states()
        upd = bool(sts) and sts[0]._updating()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        o.step()
        torch.cuda.synchronize()
        if s >= 12:
            times[upd].append((time.perf_counter() - t0) * 1e3)
    return {("update" if k else "non-update"): sorted(v)[len(v) // 2] for k, v in times.items() if v}


if __name__ == "__main__":
    main()
