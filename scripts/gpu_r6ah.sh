#!/usr/bin/env bash
# Round 6: batch-1024 A/B of the launch table before / after the stride-2 re-tune (same box).
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r6ah}
mkdir -p "$OUT"
cp faster_distributed_training_amd/ops/conv_tuned.json "$OUT/new.json"
j() { grep -h '"value"' "$OUT/$1.log" > "$OUT/$1.json"; echo "$1 $(grep -o '"ms_per_step": [0-9.]*' $OUT/$1.json)"; }
for v in old new old new; do
  cp "$OUT/$v.json" faster_distributed_training_amd/ops/conv_tuned.json 2>/dev/null || cp scripts/conv_tuned_before_r6af.json faster_distributed_training_amd/ops/conv_tuned.json
  timeout -k 10 300 python bench.py > "$OUT/bs1024_$v.log" 2>&1 || { echo "bench failed"; exit 1; }
  j bs1024_$v
done
cp "$OUT/new.json" faster_distributed_training_amd/ops/conv_tuned.json
