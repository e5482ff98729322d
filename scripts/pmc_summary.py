#!/usr/bin/env python3
"""Per-kernel counter summary of rocprofv3 --pmc passes (one directory per pass, each holding a
``*_counter_collection.csv``): for every kernel whose name matches ``--match``, the mean per
dispatch of every counter collected in any pass, plus derived ratios (MFMA busy per wave-cycle,
wait fractions, LDS bank-conflict share, L2 hit rate).

    python scripts/pmc_summary.py gpurun_out/r6b/pmc_h3 --match conv:: --out profiles/r6/pmc_h3.md
"""
import argparse
import collections
import csv
import glob
import os


def load(dirs, match):
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    dur = collections.defaultdict(list)
    for d in dirs:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            with open(f) as fh:
                for r in csv.DictReader(fh):
                    name = r["Kernel_Name"]
                    if match not in name:
                        continue
                    key = (os.path.basename(os.path.dirname(f)) if False else name, r["Grid_Size"])
                    acc[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
                    dur[key].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-3)
    return acc, dur


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("root")
    ap.add_argument("--match", default="conv::")
    ap.add_argument("--arms", default="h3,tuned")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    lines = []
    for arm in a.arms.split(","):
        dirs = sorted(glob.glob(os.path.join(a.root, f"{arm}_p*")))
        dirs = [d for d in dirs if os.path.isdir(d)]
        acc, dur = load(dirs, a.match)
        for (name, grid), cs in sorted(acc.items(), key=lambda kv: -sum(dur[kv[0]])):
            m = {k: sum(v) / len(v) for k, v in cs.items()}
            us = sorted(dur[(name, grid)])[len(dur[(name, grid)]) // 2]
            lines.append(f"## {arm}: `{name[:110]}` grid {grid}, median dispatch {us:.1f} us (counter passes)")
            for k in sorted(m):
                lines.append(f"- {k}: {m[k]:.4g}")
            wc = m.get("SQ_WAVE_CYCLES")
            if wc:
                for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS",
                          "SQ_ACTIVE_INST_VMEM", "SQ_WAIT_INST_LDS"):
                    if k in m:
                        lines.append(f"- {k} / SQ_WAVE_CYCLES: {m[k] / wc:.3f}")
            if "SQ_VALU_MFMA_BUSY_CYCLES" in m and "GRBM_GUI_ACTIVE" in m:
                lines.append(f"- MFMA busy / (GRBM_GUI_ACTIVE x 4 SIMD x 32 CU per XCD): "
                             f"{m['SQ_VALU_MFMA_BUSY_CYCLES'] / (m['GRBM_GUI_ACTIVE'] * 128):.3f}")
            if "SQ_LDS_BANK_CONFLICT" in m and m.get("SQ_LDS_IDX_ACTIVE"):
                lines.append(f"- LDS bank conflict share: {m['SQ_LDS_BANK_CONFLICT'] / m['SQ_LDS_IDX_ACTIVE']:.3f}")
            if "TCC_HIT_sum" in m and "TCC_MISS_sum" in m:
                lines.append(f"- L2 hit rate: {m['TCC_HIT_sum'] / max(1.0, m['TCC_HIT_sum'] + m['TCC_MISS_sum']):.3f}")
            lines.append("")
    txt = "\n".join(lines)
    print(txt)
    if a.out:
        os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
        with open(a.out, "w") as f:
            f.write(txt + "\n")


if __name__ == "__main__":
    main()
