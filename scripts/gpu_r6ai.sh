#!/usr/bin/env bash
# Round 6: whole-step A/B of the tap split on the halo weight gradient (batch 1024 / 128).
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r6ai}
mkdir -p "$OUT"
j() { grep -h '"value"' "$OUT/$1.log" > "$OUT/$1.json"; echo "$1 $(grep -o '"ms_per_step": [0-9.]*' $OUT/$1.json)"; }
for v in 1 2 1 2; do
  FDT_WGRAD_H3_TS=$v timeout -k 10 300 python bench.py > "$OUT/bs1024_ts$v.log" 2>&1 || { echo "bench failed"; exit 1; }
  j bs1024_ts$v
done
for v in 1 2 1 2; do
  FDT_WGRAD_H3_TS=$v timeout -k 10 300 python bench.py --global-batch 128 --steps 40 > "$OUT/bs128_ts$v.log" 2>&1 || { echo "bench failed"; exit 1; }
  j bs128_ts$v
done
