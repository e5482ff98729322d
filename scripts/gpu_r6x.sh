#!/usr/bin/env bash
# Round 6: linear weight-gradient probe + NGD rank balance sweep (simulated world-8 ranks,
# FDT_NGD_AXIS_COST variants).
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r6x}
mkdir -p "$OUT"
timeout -k 10 300 python -u scripts/linear_wgrad_probe.py > "$OUT/linear_wgrad_probe.txt" 2>&1 || { echo "probe failed"; tail -10 "$OUT/linear_wgrad_probe.txt"; exit 1; }
grep -v amdgpu.ids "$OUT/linear_wgrad_probe.txt" | sed 's/.*||/||/'
for c in 400000 100000; do
  for r in 0 1 2 3 4 5 6 7; do
    FDT_NGD_AXIS_COST=$c timeout -k 10 300 python bench.py --ngd --meta_learning --simulate-world 8 --simulate-rank $r --steps 20 --warmup 12 > "$OUT/ngd_c${c}_r$r.log" 2>&1 || { echo "sim failed"; tail -5 "$OUT/ngd_c${c}_r$r.log"; exit 1; }
    echo "axis_cost $c rank $r $(grep -ho '"ms_per_step": [0-9.]*' $OUT/ngd_c${c}_r$r.log)"
  done
done
