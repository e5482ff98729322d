#!/usr/bin/env python3
"""Calibration factors for the roofline tables from ``scripts/pmc_calib.sh``.

For every microkernel of ``tools/pmc_calib.hip`` (known bytes or MFMA FLOPs per dispatch):
  bytes per FETCH_SIZE KiB unit (16 / 8 / 4 B per lane streaming reads), bytes per WRITE_SIZE
  KiB unit, FLOP per SQ_VALU_MFMA_BUSY_CYCLES, and the effective clock GRBM_GUI_ACTIVE / 8 /
  duration of the (long, MFMA-bound) dispatch -- written as JSON for ``pmc_table.py``.

    python scripts/pmc_calib_table.py gpurun_out/pmc_calib [--out profiles/pmc/calibration.json]
"""
from __future__ import annotations

import argparse
import collections
import csv
import glob
import json
import os

GIB = 1 << 30
MFMA_FLOP = 256 * 8 * 4 * 4096 * 4 * 32768.0  # grid x waves x iters x mfma/iter x FLOP (pmc_calib.hip)
TRUE = {"read16": ("B", GIB), "read8": ("B", GIB), "read4": ("B", GIB), "write16": ("B", GIB),
        "copy16": ("B", 2 * GIB), "mfma": ("FLOP", MFMA_FLOP)}


def kind(name: str) -> str | None:
    if "read_k" in name:
        if "4u>" in name or "uint4" in name:
            return "read16"
        if "2u>" in name or "uint2" in name:
            return "read8"
        return "read4"
    for k in ("copy16", "write16", "mfma"):
        if k + "_k" in name:
            return k
    return None


def per_kernel(d, counters):
    f = glob.glob(os.path.join(d, "**", "*counter_collection.csv" if counters else "*kernel_trace.csv"),
                  recursive=True)
    assert f, f"nothing under {d}"
    out = collections.defaultdict(list)
    if counters:
        per = collections.defaultdict(lambda: collections.Counter())
        names = {}
        for r in csv.DictReader(open(f[0])):
            did = int(r["Dispatch_Id"])
            per[did][r["Counter_Name"]] += float(r["Counter_Value"])
            names[did] = r["Kernel_Name"]
        for did in sorted(per):
            k = kind(names[did])
            if k:
                out[k].append(per[did])
    else:
        for r in csv.DictReader(open(f[0])):
            k = kind(r["Kernel_Name"])
            if k:
                out[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    tm = per_kernel(os.path.join(a.dir, "time"), False)
    ctr = collections.defaultdict(lambda: collections.Counter())
    for p in sorted(glob.glob(os.path.join(a.dir, "p*"))):
        if os.path.isdir(p):
            for k, lst in per_kernel(p, True).items():
                for c in lst[1:]:  # the second (timed) dispatch of each kernel
                    ctr[k].update(c)
    res = {}
    lines = ["| kernel | true amount | duration ms | rate | FETCH_SIZE KiB | bytes / FETCH_SIZE byte | "
             "WRITE_SIZE KiB | bytes / WRITE_SIZE byte | MFMA busy cyc | FLOP / busy cyc | GRBM/8/t GHz |",
             "|---|---:|---:|---:|---:|---:|---:|---:|---:|---:|---:|"]
    for k, (unit, amount) in TRUE.items():
        t = sorted(tm.get(k, [0.0]))[len(tm.get(k, [0.0])) // 2]
        c = ctr.get(k, collections.Counter())
        fetch, write, busy, grbm = c["FETCH_SIZE"], c["WRITE_SIZE"], c["SQ_VALU_MFMA_BUSY_CYCLES"], c["GRBM_GUI_ACTIVE"]
        rd_true = amount if k.startswith("read") else (amount / 2 if k == "copy16" else 0)
        wr_true = amount if k == "write16" else (amount / 2 if k == "copy16" else 0)
        r = {"duration_s": t, "fetch_kib": fetch, "write_kib": write, "mfma_busy": busy, "grbm": grbm}
        if unit == "B":
            r["bytes"] = amount
            r["read_factor"] = rd_true / (fetch * 1024) if fetch and rd_true else None
            r["write_factor"] = wr_true / (write * 1024) if write and wr_true else None
        else:
            r["flop"] = amount
            r["flop_per_busy_cycle"] = amount / busy if busy else None
        r["eff_ghz"] = grbm / 8 / t * 1e-9 if t and grbm else None
        res[k] = r
        fmt = lambda v, p=2: "—" if v is None else f"{v:.{p}f}"  # noqa: E731
        rate = amount / t / 1e12 if t else 0
        lines.append(f"| {k} | {amount:.3e} {unit} | {t * 1e3:.3f} | {rate:.2f} {'TB/s' if unit == 'B' else 'TF/s'} | "
                     f"{fetch:.0f} | {fmt(r.get('read_factor'))} | {write:.0f} | {fmt(r.get('write_factor'))} | "
                     f"{busy:.3e} | {fmt(r.get('flop_per_busy_cycle'), 1)} | {fmt(r['eff_ghz'])} |")
    print("\n".join(lines))
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)
        with open(os.path.splitext(a.out)[0] + ".md", "w") as f:
            f.write("# Counter calibration (tools/pmc_calib.hip, scripts/pmc_calib.sh)\n\n" + "\n".join(lines) + "\n")


if __name__ == "__main__":
    main()
