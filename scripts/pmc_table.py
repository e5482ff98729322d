#!/usr/bin/env python3
"""Per-kernel roofline table from the passes of ``scripts/pmc_step.sh``.

Dispatches of the timing pass and of each counter pass are matched by
(kernel name, grid size, n-th occurrence), so a dispatch that exists in one pass only is
dropped instead of shifting the alignment.  Columns (per step = totals / --steps):

  ms      kernel time (timing pass, no counters attached)
  rdGB    FETCH_SIZE x the calibrated bytes per FETCH_SIZE byte of a 16-B/lane stream
          (profiles/pmc/calibration.json, tools/pmc_calib.hip: 2.0 on gfx950 for coalesced
          16-, 8- and 4-B/lane streams alike -- FETCH_SIZE tallies a 128-B request at 64 B); a
          row whose traffic would then exceed the achievable 6.3 TB/s cannot be made of full
          128-B requests and is reported at factor 1 instead (marked "n": 64-B requests,
          tallied at their size -- the lower bound of its bytes); memory-side, Infinity-Cache
          hits included
  wrGB    WRITE_SIZE x its calibrated factor
  TB/s    (rdGB + wrGB) / ms
  TF/s    SQ_VALU_MFMA_BUSY_CYCLES x the calibrated FLOP per busy cycle (1024 for
          32x32x16 bf16: 32 busy cycles per 32768-FLOP MFMA, measured by the MFMA loop) / ms
  mfma%   MFMA busy cycles / (kernel time x 2.4 GHz x 1024 SIMDs): the fraction of the
          peak-clock MFMA rate (GRBM_GUI_ACTIVE / 8 reads high on dispatches shorter than
          ~0.3 ms, so it is not used as the cycle base)
  ldsc%   SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE
  roof%   max(bytes / 6.3 TB/s, FLOP / 2.5 PF) / measured time
  GHz     per-row clock: (GRBM_GUI_ACTIVE / 8 - fitted window overhead x calls) / the same
          pass's kernel time.  GRBM_GUI_ACTIVE counts a counter window that opens before and
          closes after each dispatch, so raw GRBM / time reads above the 2.4 GHz peak on short
          dispatches; a least-squares fit of cycles = clock x time + overhead over every
          dispatch of the GRBM pass gives the clock and the per-dispatch window overhead
          (header line).  Shown to one decimal (the fit residual is a few 0.01 GHz) for rows
          whose dispatches average >= 0.1 ms.

    python scripts/pmc_table.py gpurun_out/pmc_x_1024 --steps 4 [--out profiles/x.md]
"""
from __future__ import annotations

import argparse
import collections
import csv
import glob
import json
import os
import re

HBM = 6.3e12
MFMA = 2.5e15
PEAK_GHZ = 2.4
CALIB = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "profiles", "pmc",
                     "calibration.json")


def calibration():
    """(read factor of full-line streams, read factor of 64-B requests, write factor, FLOP per
    MFMA busy cycle)."""
    f16, fn, fw, fl = 2.0, 1.0, 1.0, 1024.0
    if os.path.exists(CALIB):
        c = json.load(open(CALIB))
        f16 = c.get("read16", {}).get("read_factor") or f16
        fw = c.get("write16", {}).get("write_factor") or fw
        fl = c.get("mfma", {}).get("flop_per_busy_cycle") or fl
    return f16, fn, fw, fl


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


def clock_fit(d):
    """(clock Hz, window overhead cycles per dispatch, {key: same-pass kernel time}) from the
    counter pass holding GRBM_GUI_ACTIVE, or None."""
    import numpy as np
    for p in sorted(glob.glob(os.path.join(d, "p*"))):
        if not os.path.isdir(p):
            continue
        c = load_pmc(p)
        if not any("GRBM_GUI_ACTIVE" in v for v in c.values()):
            continue
        t = load_time(p)
        ks = [k for k, v in c.items() if k in t and "GRBM_GUI_ACTIVE" in v]
        x = np.array([t[k] for k in ks])
        y = np.array([c[k]["GRBM_GUI_ACTIVE"] / 8 for k in ks])
        (a, b), *_ = np.linalg.lstsq(np.stack([x, np.ones_like(x)], 1), y, rcond=None)
        return a, b, {k: t[k] for k in ks}
    return None


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
    fit = clock_fit(a.dir)
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
            if fit and k in fit[2]:
                g["t_grbm"] += fit[2][k]
                g["n_grbm"] += 1
    S = a.steps
    rows = []
    tot_t = sum(g["t"] for g in agg.values()) / S
    f16, fnar, fw, fpc = calibration()
    for (name, grid), g in agg.items():
        t = g["t"] / S
        wr = fw * g["WRITE_SIZE"] * 1024 / S
        rd = f16 * g["FETCH_SIZE"] * 1024 / S
        narrow = t > 0 and (rd + wr) / t > HBM
        if narrow:
            rd = fnar * g["FETCH_SIZE"] * 1024 / S
        flop = g["SQ_VALU_MFMA_BUSY_CYCLES"] * fpc / S
        mf = g["SQ_VALU_MFMA_BUSY_CYCLES"] / S / (t * PEAK_GHZ * 1e9 * 1024) if t else 0.0
        per_call = t / max(g["calls"] / S, 1e-9)
        ghz = None
        if fit and g["t_grbm"] and g["t_grbm"] / g["n_grbm"] >= 1e-4:
            ghz = (g["GRBM_GUI_ACTIVE"] / 8 - fit[1] * g["n_grbm"]) / g["t_grbm"] * 1e-9
        ldsc = g["SQ_LDS_BANK_CONFLICT"] / g["SQ_LDS_IDX_ACTIVE"] if g["SQ_LDS_IDX_ACTIVE"] else 0.0
        roof = max((rd + wr) / HBM, flop / MFMA)
        rows.append((t, name + (" n" if narrow else ""), grid, g["calls"] / S, rd, wr, flop, mf, ldsc, roof, ghz))
    rows.sort(reverse=True)
    lines = [f"# per-kernel roofline ({a.dir}, {S} steps)", "",
             "Eager launches (scripts/pmc_step.sh runs bench.py --no-graphs so each dispatch is "
             "counted on its own); the graph-replayed step additionally folds the 1x1-conv "
             "residual joins (FDT_JOIN_FOLD) and is a few % faster.", "",
             f"total kernel time {tot_t * 1e3:.3f} ms/step; rdGB = FETCH_SIZE x {f16:.2f} (calibrated 16-B stream; "
             f"'n' rows: x {fnar:.2f}, 64-B requests); TF/s = MFMA busy x {fpc:.0f}; mfma% at {PEAK_GHZ} GHz; "
             "roof% = max(bytes/6.3TB/s, FLOP/2.5PF)/time",
             "",
             (f"clock fit over {len(fit[2])} dispatches of the GRBM pass: {fit[0] * 1e-9:.3f} GHz + "
              f"{fit[1]:.0f} cycles ({fit[1] / fit[0] * 1e6:.1f} us) of counter window per dispatch"
              if fit else "no GRBM pass"),
             "",
             "| ms/step | calls | kernel | grid | rdGB | wrGB | TB/s | TF/s | mfma% | ldsc% | roof% | GHz |",
             "|---:|---:|---|---:|---:|---:|---:|---:|---:|---:|---:|---:|"]
    sum_roof = 0.0
    for t, name, grid, calls, rd, wr, flop, mf, ldsc, roof, ghz in rows:
        sum_roof += roof
    for t, name, grid, calls, rd, wr, flop, mf, ldsc, roof, ghz in rows[: a.top]:
        lines.append(f"| {t * 1e3:.3f} | {calls:.1f} | `{name}` | {grid} | {rd / 1e9:.3f} | {wr / 1e9:.3f} | "
                     f"{(rd + wr) / t / 1e12:.2f} | {flop / t / 1e12:.0f} | {mf * 100:.1f} | {ldsc * 100:.1f} | "
                     f"{roof / t * 100:.0f} | {'—' if ghz is None else f'{ghz:.1f}'} |")
    lines += ["", f"sum of per-kernel roofline bounds {sum_roof * 1e3:.3f} ms/step vs measured {tot_t * 1e3:.3f} ms/step "
              f"({sum_roof / tot_t * 100:.0f} % of roofline overall)"]
    txt = "\n".join(lines)
    print(txt)
    if a.out:
        with open(a.out, "w") as f:
            f.write(txt + "\n")


if __name__ == "__main__":
    main()
