#!/usr/bin/env python3
"""Per-dispatch timeline of one training step from a rocprofv3 kernel trace (csv):
kernel, workgroups, duration and the idle gap before it, in launch order.

    python scripts/ktrace_step.py RUN_kernel_trace.csv [--step -2] [--marker madgrad_kernel]

Steps are delimited by the optimizer kernel (``--marker``, one launch per step); ``--step``
picks one (python index over the complete steps, default the second to last)."""
import argparse
import csv
import re


def short(name, n=70):
    name = re.sub(r"\(.*", "", name)
    name = name.replace("void ", "").replace("fdt::", "")
    return name[:n]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--step", type=int, default=-2)
    ap.add_argument("--marker", default="madgrad_kernel")
    ap.add_argument("--min-us", type=float, default=0.0)
    a = ap.parse_args()
    rows = []
    with open(a.trace) as f:
        for r in csv.DictReader(f):
            wg = 1
            for ax in "XYZ":
                wg *= max(1, int(r[f"Grid_Size_{ax}"]) // max(1, int(r[f"Workgroup_Size_{ax}"])))
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], wg,
                         int(r["VGPR_Count"]) + int(r["Accum_VGPR_Count"]), int(r["LDS_Block_Size"])))
    rows.sort()
    ends = [i for i, r in enumerate(rows) if a.marker in r[2]]
    if len(ends) < 2:
        raise SystemExit(f"fewer than two '{a.marker}' launches in the trace")
    spans = list(zip(ends[:-1], ends[1:]))
    lo, hi = spans[a.step]
    step = rows[lo + 1:hi + 1]
    t0 = step[0][0]
    busy = sum(e - s for s, e, *_ in step)
    wall = step[-1][1] - rows[lo][1]
    print(f"step: {len(step)} kernels, wall {wall / 1e3:.1f} us, busy {busy / 1e3:.1f} us, "
          f"idle {(wall - busy) / 1e3:.1f} us")
    prev_end = rows[lo][1]
    for s, e, name, wg, vgpr, lds in step:
        dur = (e - s) / 1e3
        if dur >= a.min_us:
            print(f"{(s - t0) / 1e3:9.1f} {dur:8.1f} us gap {max(0, s - prev_end) / 1e3:6.1f}  wg {wg:6d} "
                  f"v{vgpr:3d} lds {lds:6d}  {short(name)}")
        prev_end = max(prev_end, e)


if __name__ == "__main__":
    main()
