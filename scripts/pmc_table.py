#!/usr/bin/env python3
"""Per-kernel roofline table from the passes of ``scripts/pmc_step.sh``.

Dispatches of the timing pass and of each counter pass are matched by
(kernel name, grid size, n-th occurrence), so a dispatch that exists in one pass only is
dropped instead of shifting the alignment.  Columns (per step = totals / --steps):

  ms      kernel time (timing pass, no counters attached)
  rdGB    2 x FETCH_SIZE  (gfx950 FETCH_SIZE counts half the bytes of a 16-B/lane stream,
          MI355X_MICROARCH.md "HBM"); memory-side, Infinity-Cache hits included
  wrGB    WRITE_SIZE
  TB/s    (rdGB + wrGB) / ms
  TF/s    SQ_VALU_MFMA_BUSY_CYCLES x 1024 FLOP (= 32 busy cycles per 32x32x16 bf16 MFMA of
          32*32*16*2 FLOP) / ms
  mfma%   MFMA busy cycles / (GRBM_GUI_ACTIVE/8 cycles x 1024 SIMDs)
  ldsc%   SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE
  roof%   max(bytes / 6.3 TB/s, FLOP / 2.5 PF) / measured time

    python scripts/pmc_table.py gpurun_out/pmc_x_1024 --steps 4 [--out profiles/x.md]
"""
from __future__ import annotations

import argparse
import collections
import csv
import glob
import os
import re

HBM = 6.3e12
MFMA = 2.5e15


def _short(name: str) -> str:
    name = re.sub(r"\(.*$", "", name) if "(fdt::" in name or name.endswith(")") else name
    name = name.replace("void ", "").replace("fdt::", "").replace("__hip_bfloat16", "bf16")
    return name[:70]


def _grid(r):
    if "Grid_Size" in r:
        return int(r["Grid_Size"])
    return int(r.get("Grid_Size_X", 1)) * int(r.get("Grid_Size_Y", 1)) * int(r.get("Grid_Size_Z", 1))


def load_time(d):
    f = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
    assert f, f"no kernel trace under {d}"
    rows = sorted(csv.DictReader(open(f[0])), key=lambda r: int(r["Dispatch_Id"]))
    seen = collections.Counter()
    out = {}
    for r in rows:
        k = (r["Kernel_Name"], _grid(r))
        out[k + (seen[k],)] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
        seen[k] += 1
    return out


def load_pmc(d):
    f = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    assert f, f"no counter csv under {d}"
    per = collections.defaultdict(dict)
    meta = {}
    for r in csv.DictReader(open(f[0])):
        did = int(r["Dispatch_Id"])
        per[did][r["Counter_Name"]] = per[did].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        meta[did] = (r["Kernel_Name"], _grid(r))
    seen = collections.Counter()
    out = {}
    for did in sorted(per):
        k = meta[did]
        out[k + (seen[k],)] = per[did]
        seen[k] += 1
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--steps", type=int, default=4)
    ap.add_argument("--top", type=int, default=40)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    tm = load_time(os.path.join(a.dir, "time"))
    ctr = collections.defaultdict(dict)
    for p in sorted(glob.glob(os.path.join(a.dir, "p*"))):
        if os.path.isdir(p):
            for k, v in load_pmc(p).items():
                ctr[k].update(v)
    agg = collections.defaultdict(lambda: collections.Counter())
    for k, t in tm.items():
        name, grid, _ = k
        g = agg[(_short(name), grid)]
        g["calls"] += 1
        g["t"] += t
        c = ctr.get(k)
        if c:
            g["matched"] += 1
            for n, v in c.items():
                g[n] += v
    S = a.steps
    rows = []
    tot_t = sum(g["t"] for g in agg.values()) / S
    for (name, grid), g in agg.items():
        t = g["t"] / S
        rd = 2 * g["FETCH_SIZE"] * 1024 / S
        wr = g["WRITE_SIZE"] * 1024 / S
        flop = g["SQ_VALU_MFMA_BUSY_CYCLES"] * 1024 / S
        cyc = g["GRBM_GUI_ACTIVE"] / 8 / S
        mf = g["SQ_VALU_MFMA_BUSY_CYCLES"] / S / (cyc * 1024) if cyc else 0.0
        ldsc = g["SQ_LDS_BANK_CONFLICT"] / g["SQ_LDS_IDX_ACTIVE"] if g["SQ_LDS_IDX_ACTIVE"] else 0.0
        roof = max((rd + wr) / HBM, flop / MFMA)
        rows.append((t, name, grid, g["calls"] / S, rd, wr, flop, mf, ldsc, roof, cyc / t * 1e-9 if t and cyc else 0))
    rows.sort(reverse=True)
    lines = [f"# per-kernel roofline ({a.dir}, {S} steps)", "",
             f"total kernel time {tot_t * 1e3:.3f} ms/step; rdGB = 2 x FETCH_SIZE; roof% = max(bytes/6.3TB/s, FLOP/2.5PF)/time",
             "",
             "| ms/step | calls | kernel | grid | rdGB | wrGB | TB/s | TF/s | mfma% | ldsc% | roof% | GHz |",
             "|---:|---:|---|---:|---:|---:|---:|---:|---:|---:|---:|---:|"]
    sum_roof = 0.0
    for t, name, grid, calls, rd, wr, flop, mf, ldsc, roof, ghz in rows:
        sum_roof += roof
    for t, name, grid, calls, rd, wr, flop, mf, ldsc, roof, ghz in rows[: a.top]:
        lines.append(f"| {t * 1e3:.3f} | {calls:.1f} | `{name}` | {grid} | {rd / 1e9:.3f} | {wr / 1e9:.3f} | "
                     f"{(rd + wr) / t / 1e12:.2f} | {flop / t / 1e12:.0f} | {mf * 100:.1f} | {ldsc * 100:.1f} | "
                     f"{roof / t * 100:.0f} | {ghz:.2f} |")
    lines += ["", f"sum of per-kernel roofline bounds {sum_roof * 1e3:.3f} ms/step vs measured {tot_t * 1e3:.3f} ms/step "
              f"({sum_roof / tot_t * 100:.0f} % of roofline overall)"]
    txt = "\n".join(lines)
    print(txt)
    if a.out:
        with open(a.out, "w") as f:
            f.write(txt + "\n")


if __name__ == "__main__":
    main()
