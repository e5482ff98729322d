#!/usr/bin/env python3
"""GPU busy fraction of the last K steps of a kernel trace: union of kernel intervals between
consecutive optimizer-marker kernels (one per step) over the wall span they cover.

    python scripts/busy_fraction.py RUN_kernel_trace.csv --marker sgd_kernel --steps 10
"""
import argparse
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--marker", default="sgd_kernel")
    ap.add_argument("--steps", type=int, default=10)
    a = ap.parse_args()
    rows = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"])
                   for r in csv.DictReader(open(a.trace))), key=lambda t: t[0])
    marks = [e for s, e, n in rows if a.marker in n]
    assert len(marks) > a.steps, f"only {len(marks)} marker kernels"
    t0, t1 = marks[-a.steps - 1], marks[-1]
    busy, cur_s, cur_e = 0, None, None
    for s, e, _ in rows:
        if e <= t0 or s >= t1:
            continue
        s, e = max(s, t0), min(e, t1)
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        busy += cur_e - cur_s
    wall = t1 - t0
    print(f"{a.steps} steps: wall {wall / 1e6 / a.steps:.3f} ms/step, GPU busy {busy / 1e6 / a.steps:.3f} ms/step "
          f"({100.0 * busy / wall:.1f} %), idle {100.0 * (1 - busy / wall):.1f} %")


if __name__ == "__main__":
    main()
