#!/usr/bin/env python3
"""Markdown table of the NGD projection kernels' counters from scripts/pmc_ngd.sh output.

    python scripts/pmc_ngd_table.py gpurun_out/<tag>/p1 > profiles/pmc/ngd_proj_counters.md
"""
import collections
import csv
import glob
import sys

f = glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)[0]
acc = collections.defaultdict(collections.Counter)
for r in csv.DictReader(open(f)):
    n = r["Kernel_Name"]
    if "proj" not in n:
        continue
    key = (n.split("(")[0].replace("fdt::", "").replace("void ", ""), r.get("Grid_Size", r.get("Grid_Size_X")))
    acc[key][r["Counter_Name"]] += float(r["Counter_Value"])
print("# NGD projection kernels, transformer parameter set (scripts/pmc_ngd.sh)\n")
print("Fractions of SQ_WAVE_CYCLES; 16 optimizer steps (init schedule included).\n")
print("| kernel | grid (threads) | VALU active | LDS active | wait LDS | wait any | VALU insts | LDS insts |")
print("|---|---:|---:|---:|---:|---:|---:|---:|")
for k, c in sorted(acc.items(), key=lambda kv: -kv[1]["SQ_WAVE_CYCLES"]):
    wc = c["SQ_WAVE_CYCLES"] or 1.0
    print(f"| `{k[0]}` | {k[1]} | {c['SQ_ACTIVE_INST_VALU'] / wc:.2f} | {c['SQ_ACTIVE_INST_LDS'] / wc:.2f} | "
          f"{c['SQ_WAIT_INST_LDS'] / wc:.2f} | {c['SQ_WAIT_ANY'] / wc:.2f} | {c['SQ_INSTS_VALU']:.3g} | "
          f"{c['SQ_INSTS_LDS']:.3g} |")
