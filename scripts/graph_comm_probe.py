#!/usr/bin/env python3
"""HIP-graph semantics probe for the DDP overlap design (round 4).

Answers, on the MI355X box, the questions that decide how bucket all-reduces are issued
while the engine's backward is a HIP graph:

 1. Does a graph replay run two forked branches concurrently?   (capture RCCL inside)
 2. Does an external event record node inside a graph fire mid-replay, so another stream
    (RCCL's) can start when the node is reached instead of at graph end?
 3. What does an external event-record node cost on the compute timeline, against a
    graph boundary (two graphs launched back to back)?
 4. Can a world-1 RCCL all-reduce be captured inside a graph on a forked stream?

Spin kernels are torch.cuda._sleep (one thread, clock-based).  Prints one line per probe.
"""
import os
import time

import torch


def ms(a, b):
    return a.elapsed_time(b)


def calib():
    torch.cuda._sleep(1000)
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    torch.cuda._sleep(10_000_000)
    e.record()
    torch.cuda.synchronize()
    per = ms(s, e) / 10_000_000
    return int(1.0 / per)  # cycles per ms


def probe_branches(cyc):
    g = torch.cuda.CUDAGraph()
    side = torch.cuda.Stream()
    with torch.cuda.graph(g):
        cur = torch.cuda.current_stream()
        side.wait_stream(cur)
        torch.cuda._sleep(cyc)
        with torch.cuda.stream(side):
            torch.cuda._sleep(cyc)
        cur.wait_stream(side)
    g.replay()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(5):
        g.replay()
    e.record()
    torch.cuda.synchronize()
    t = ms(s, e) / 5
    print(f"[1] forked branches of 1.0 ms each: replay {t:.3f} ms -> {'CONCURRENT' if t < 1.5 else 'SERIALISED'}",
          flush=True)


def probe_external_event(cyc):
    try:
        ev = torch.cuda.Event(external=True)
        ev.record()
    except RuntimeError as e:  # torch on ROCm refuses external events
        print(f"[2] external event record nodes: unavailable ({e})", flush=True)
        _probe_in_graph_fork(cyc)
        return
    ev = torch.cuda.Event(external=True)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        torch.cuda._sleep(cyc)          # A: 1 ms
        ev.record()
        torch.cuda._sleep(2 * cyc)      # B: 2 ms
    g.replay()
    torch.cuda.synchronize()
    other = torch.cuda.Stream(priority=-1)
    res = []
    for _ in range(3):
        s = torch.cuda.Event(enable_timing=True)
        e_other = torch.cuda.Event(enable_timing=True)
        e_main = torch.cuda.Event(enable_timing=True)
        s.record()
        g.replay()
        e_main.record()
        with torch.cuda.stream(other):
            other.wait_event(ev)
            e_other.record(other)
        torch.cuda.synchronize()
        res.append((ms(s, e_other), ms(s, e_main)))
    t_o, t_m = res[-1]
    verdict = "MID-GRAPH (fires at the node)" if 0.7 < t_o < 1.6 else ("AT GRAPH END" if t_o > 2.5 else "NO WAIT")
    print(f"[2] external event: other stream released after {t_o:.3f} ms, graph done {t_m:.3f} ms -> {verdict}",
          flush=True)
    _probe_in_graph_fork(cyc)


def _probe_in_graph_fork(cyc):
    # A wait captured in the SAME graph on a forked stream (no host involvement)
    g2 = torch.cuda.CUDAGraph()
    side = torch.cuda.Stream()
    ev2 = torch.cuda.Event()
    flag = torch.zeros(1, device="cuda")
    with torch.cuda.graph(g2):
        cur = torch.cuda.current_stream()
        torch.cuda._sleep(cyc)
        ev2.record()
        with torch.cuda.stream(side):
            side.wait_event(ev2)
            torch.cuda._sleep(cyc)
            flag.add_(1)
        torch.cuda._sleep(2 * cyc)
        cur.wait_stream(side)
    g2.replay()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    g2.replay()
    e.record()
    torch.cuda.synchronize()
    t = ms(s, e)
    print(f"[2b] in-graph fork after A (A 1 ms, then B 2 ms || C 1 ms): replay {t:.3f} ms "
          f"-> {'CONCURRENT' if t < 3.5 else 'SERIALISED'}", flush=True)


def probe_costs():
    x = torch.zeros(1024, device="cuda")
    n = 200

    def body(k_events, evs):
        for i in range(n):
            x.add_(1.0)
            if k_events and i % (n // k_events) == n // k_events - 1:
                evs[i // (n // k_events)].record()

    res = {}
    for k in (0,):
        evs = []
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            body(k, evs)
        g.replay()
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(20):
            g.replay()
        e.record()
        torch.cuda.synchronize()
        res[k] = ms(s, e) / 20 * 1e3
    # the same 200 kernels as 11 graphs launched back to back
    graphs = []
    for j in range(11):
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for _ in range(n // 11 + (1 if j < n % 11 else 0)):
                x.add_(1.0)
        graphs.append(g)
    for g in graphs:
        g.replay()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(20):
        for g in graphs:
            g.replay()
    e.record()
    torch.cuda.synchronize()
    t_split = ms(s, e) / 20 * 1e3
    # host time per replay of the split version
    t0 = time.perf_counter()
    for _ in range(20):
        for g in graphs:
            g.replay()
    host = (time.perf_counter() - t0) / 20 * 1e6
    torch.cuda.synchronize()
    print(f"[3] 200 tiny kernels: one graph {res[0]:.1f} us, as 11 graphs {t_split:.1f} us "
          f"({(t_split - res[0]) / 10:.2f} us per boundary; host {host:.1f} us)", flush=True)


def probe_rccl_capture(cyc):
    import torch.distributed as dist
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29533")
    os.environ.setdefault("TORCH_NCCL_HIGH_PRIORITY", "1")
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    buf = torch.ones(4 << 20, device="cuda")
    dist.all_reduce(buf)  # warm the communicator
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    side = torch.cuda.Stream()
    try:
        with torch.cuda.graph(g):
            cur = torch.cuda.current_stream()
            buf.mul_(2.0)
            side.wait_stream(cur)
            with torch.cuda.stream(side):
                dist.all_reduce(buf)
            torch.cuda._sleep(cyc)
            cur.wait_stream(side)
        buf.fill_(1.0)
        g.replay()
        torch.cuda.synchronize()
        ok = bool((buf == 2.0).all().item())
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(5):
            g.replay()
        e.record()
        torch.cuda.synchronize()
        print(f"[4] RCCL all-reduce captured on a forked stream: value ok={ok}, replay {ms(s, e) / 5:.3f} ms "
              f"(sleep branch 1.0 ms)", flush=True)
        # the DDP pattern: compute A, all-reduce of A's output on a side branch (async_op +
        # wait() joined at the END), more compute B on the main branch
        big = torch.ones(16 << 20, device="cuda")
        g3 = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g3):
            big.mul_(3.0)                      # A
            w = dist.all_reduce(big, async_op=True)
            torch.cuda._sleep(cyc)             # B (1 ms) on the main branch
            w.wait()                           # join before the capture ends
        big.fill_(1.0)
        g3.replay()
        torch.cuda.synchronize()
        ok3 = bool((big == 3.0).all().item())
        s.record()
        for _ in range(5):
            g3.replay()
        e.record()
        torch.cuda.synchronize()
        t3 = ms(s, e) / 5
        # alone: the all-reduce of 64 MB
        s.record()
        for _ in range(5):
            dist.all_reduce(big)
        e.record()
        torch.cuda.synchronize()
        tar = ms(s, e) / 5
        print(f"[5] async all_reduce captured + wait() at the end: value ok={ok3}, replay {t3:.3f} ms "
              f"(sleep 1.0 ms + all-reduce alone {tar:.3f} ms -> {'OVERLAPPED' if t3 < 1.0 + 0.5 * tar else 'SERIAL'})",
              flush=True)
    except Exception as ex:  # noqa: BLE001
        print(f"[4] RCCL capture failed: {type(ex).__name__}: {ex}", flush=True)
    dist.destroy_process_group()


def main():
    torch.cuda.init()
    cyc = calib()
    print(f"calibration: {cyc} sleep cycles per ms", flush=True)
    probe_branches(cyc)
    probe_external_event(cyc)
    probe_costs()
    probe_rccl_capture(cyc)


if __name__ == "__main__":
    main()
