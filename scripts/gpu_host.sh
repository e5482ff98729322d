#!/usr/bin/env bash
# Host submission time vs device time per step (is the step host-bound?).
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/${1:-host}
mkdir -p "$OUT"
for spec in "128 3" "128 30" "1024 3" "256 3"; do
  set -- $spec
  timeout -k 10 300 python bench.py --global-batch $1 --steps $2 --warmup 5 > "$OUT/b$1_$2.log" 2>&1 || { tail "$OUT/b$1_$2.log"; exit 1; }
  echo "bs$1 steps$2 $(grep -o '"ms_per_step": [0-9.]*' "$OUT/b$1_$2.log") $(grep -o '"host_ms_per_step": [0-9.]*' "$OUT/b$1_$2.log")"
done
timeout -k 10 300 python bench.py --model transformer --global-batch 32 --steps 10 --warmup 12 > "$OUT/tr32.log" 2>&1 || { tail "$OUT/tr32.log"; exit 1; }
echo "tr32 $(grep -o '"ms_per_step": [0-9.]*' "$OUT/tr32.log") $(grep -o '"host_ms_per_step": [0-9.]*' "$OUT/tr32.log")"
