#!/usr/bin/env python3
"""Summarise a rocprofv3 ``*_kernel_stats.csv``: per-step ms and calls of the top kernels.

    python scripts/kstats.py gpurun_out/x/prof/run_kernel_stats.csv --steps 20 [--top 25]
"""
import argparse
import csv

ap = argparse.ArgumentParser()
ap.add_argument("csv")
ap.add_argument("--steps", type=int, default=1)
ap.add_argument("--top", type=int, default=25)
a = ap.parse_args()
rows = list(csv.DictReader(open(a.csv)))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
ncall = sum(int(r["Calls"]) for r in rows)
print(f"total kernel time {tot / 1e6 / a.steps:.3f} ms/step over {a.steps} steps, {ncall / a.steps:.1f} launches/step")
for r in rows[: a.top]:
    print(f"{float(r['TotalDurationNs']) / 1e6 / a.steps:8.3f} ms/step {int(r['Calls']) / a.steps:7.1f} calls/step  "
          f"{r['Name'][:110]}")
