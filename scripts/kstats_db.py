#!/usr/bin/env python3
"""Per-step kernel statistics from a rocprofv3 rocpd database (``--kernel-trace`` default output):
the steady-state step is the interval between two consecutive launches of a once-per-step marker
kernel (the optimizer's), averaged over the last ``--steps`` such intervals; prints launches per
step, device time per step and the top kernels.

    python scripts/kstats_db.py gpurun_out/x/kt_bs128/kt_results.db --marker madgrad --steps 10
"""
import argparse
import collections
import sqlite3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--marker", default="madgrad")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--top", type=int, default=40)
    a = ap.parse_args()
    cur = sqlite3.connect(a.db).cursor()
    rows = cur.execute("select name, start, end from kernels order by start").fetchall()
    marks = [i for i, r in enumerate(rows) if a.marker in r[0]]
    if len(marks) < 2:
        raise SystemExit(f"fewer than two '{a.marker}' launches")
    marks = marks[-(a.steps + 1):]
    n = len(marks) - 1
    per = collections.defaultdict(lambda: [0, 0.0])
    launches = 0
    for i0, i1 in zip(marks, marks[1:]):
        for name, s, e in rows[i0 + 1:i1 + 1]:
            per[name][0] += 1
            per[name][1] += (e - s) * 1e-6
            launches += 1
    span = (rows[marks[-1]][1] - rows[marks[0]][1]) * 1e-6 / n
    busy = sum(v[1] for v in per.values()) / n
    print(f"{launches / n:.1f} launches/step, kernel time {busy:.3f} ms/step, marker-to-marker span {span:.3f} ms/step "
          f"(last {n} steps)")
    for name, (c, t) in sorted(per.items(), key=lambda kv: -kv[1][1])[:a.top]:
        print(f"{t / n:8.3f} ms/step {c / n:7.1f} calls/step  {name[:110]}")


if __name__ == "__main__":
    main()
