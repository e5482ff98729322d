#!/usr/bin/env python3
"""Instruction mix per basic block of one kernel in a hipcc -S output (register / VALU audit).

    python scripts/asm_mix.py file.s <mangled-name-substring>
"""
import collections
import re
import sys

s = open(sys.argv[1]).read()
names = re.findall(r"^(_ZN[A-Za-z0-9_]*):", s, re.M)
name = [n for n in names if sys.argv[2] in n][0]
i = s.index(name + ":")
j = s.index(".Lfunc_end", i)
body = s[i:j]
print(name)
blocks = re.split(r"\n(\.LBB\d+_\d+):", body)
for k in range(0, len(blocks), 2):
    lab = blocks[k - 1] if k else "entry"
    txt = blocks[k]
    ins = [l.strip().split()[0] for l in txt.split("\n") if l.strip() and not l.strip().startswith((".", ";", "_Z"))]
    c = collections.Counter()
    for x in ins:
        if x.startswith("v_mfma"):
            c["mfma"] += 1
        elif x.startswith("v_"):
            c["valu"] += 1
        elif x.startswith("s_waitcnt"):
            c["wait"] += 1
        elif x.startswith("s_barrier"):
            c["barrier"] += 1
        elif x.startswith("s_"):
            c["salu"] += 1
        elif x.startswith("ds_"):
            c["lds"] += 1
        elif x.startswith(("buffer_", "global_", "scratch_")):
            c["vmem"] += 1
    if len(ins) > 20:
        print(f"{lab:>12} {len(ins):5d} {dict(c)}")
m = re.search(r"\.vgpr_count:\s+(\d+)", s[j:j + 20000])
