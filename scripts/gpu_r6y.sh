#!/usr/bin/env bash
# Round 6: NGD rank-balance sweep, same box back to back (simulated world-8 ranks of ResNet-50
# NGD + meta-mixup, and the transformer's sharded NGD ranks at B=32).
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r6y}
mkdir -p "$OUT"
for c in 200000 400000 300000 200000 400000; do
  line="axis_cost $c:"
  for r in 0 1 2 3 4 5 6 7; do
    FDT_NGD_AXIS_COST=$c timeout -k 10 300 python bench.py --ngd --meta_learning --simulate-world 8 --simulate-rank $r --steps 20 --warmup 12 > "$OUT/ngd_c${c}_r$r.log" 2>&1 || { echo "sim failed"; tail -5 "$OUT/ngd_c${c}_r$r.log"; exit 1; }
    line="$line $(grep -ho '"ms_per_step": [0-9.]*' $OUT/ngd_c${c}_r$r.log | cut -d' ' -f2)"
  done
  echo "$line"
done
for c in 200000 400000; do
  line="transformer axis_cost $c:"
  for r in 0 1 2 3 4 5 6 7; do
    FDT_NGD_AXIS_COST=$c timeout -k 10 300 python bench.py --model transformer --simulate-world 8 --simulate-rank $r --steps 30 --warmup 15 > "$OUT/tr_c${c}_r$r.log" 2>&1 || { echo "sim failed"; tail -5 "$OUT/tr_c${c}_r$r.log"; exit 1; }
    line="$line $(grep -ho '"ms_per_step": [0-9.]*' $OUT/tr_c${c}_r$r.log | cut -d' ' -f2)"
  done
  echo "$line"
done
