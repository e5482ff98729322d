#!/usr/bin/env bash
# Round 6: whole-step A/B of the conv epilogues' write-through stores (FDT_CONV_WT).
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r6ak}
mkdir -p "$OUT"
j() { grep -h '"value"' "$OUT/$1.log" > "$OUT/$1.json"; echo "$1 $(grep -o '"ms_per_step": [0-9.]*' $OUT/$1.json)"; }
for v in 1 0 1 0; do
  FDT_CONV_WT=$v timeout -k 10 300 python bench.py > "$OUT/bs1024_wt$v.log" 2>&1 || { echo "bench failed"; exit 1; }
  j bs1024_wt$v
done
for v in 1 0; do
  FDT_CONV_WT=$v timeout -k 10 300 python bench.py --global-batch 128 --steps 40 > "$OUT/bs128_wt$v.log" 2>&1 || { echo "bench failed"; exit 1; }
  j bs128_wt$v
done
