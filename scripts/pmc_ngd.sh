#!/usr/bin/env bash
# VALU / LDS / wait counters of the NGD projection kernels (transformer parameter set).
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${1:-pmc_ngd}
mkdir -p "$OUT"
timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv -d "$OUT/p1" -o run --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_LDS -- python3 scripts/bench_ngd.py --model transformer --steps 16 > "$OUT/p1.log" 2>&1 || { echo pmc failed; tail "$OUT/p1.log"; exit 1; }
python3 - "$OUT/p1" <<'PY'
import csv, glob, sys, collections
f = glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)[0]
acc = collections.defaultdict(lambda: collections.Counter())
for r in csv.DictReader(open(f)):
    n = r["Kernel_Name"]
    if "proj" not in n:
        continue
    key = (n.split("(")[0].replace("fdt::", ""), r.get("Grid_Size", r.get("Grid_Size_X")))
    acc[key][r["Counter_Name"]] += float(r["Counter_Value"])
for k, c in sorted(acc.items()):
    wc = c["SQ_WAVE_CYCLES"] or 1
    print(k, "valu/wave-cyc %.2f lds/wave-cyc %.2f waitlds %.2f waitany %.2f insts valu %.3g lds %.3g" % (
        c["SQ_ACTIVE_INST_VALU"] / wc, c["SQ_ACTIVE_INST_LDS"] / wc, c["SQ_WAIT_INST_LDS"] / wc,
        c["SQ_WAIT_ANY"] / wc, c["SQ_INSTS_VALU"], c["SQ_INSTS_LDS"]))
PY
