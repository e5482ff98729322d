#!/usr/bin/env bash
# Round 4: switch A/B at HEAD (retuned table): fused wgrad reduce, join fold width, wgrad stages, K groups.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r4w}
mkdir -p "$OUT"
run() {
  local name=$1; shift
  timeout -k 10 300 python bench.py "$@" > "$OUT/$name.log" 2>&1 || { echo "$name failed"; tail -5 "$OUT/$name.log"; exit 1; }
  grep -h '"value"' "$OUT/$name.log" > "$OUT/$name.json"
  echo "$name $(grep -o '"ms_per_step": [0-9.]*' "$OUT/$name.json")"
}
run b1024_base --steps 30 --warmup 8
FDT_WG_FUSED_REDUCE=1 run b1024_wgfr --steps 30 --warmup 8
FDT_JOIN_FOLD_MAX=128 run b1024_fold128 --steps 30 --warmup 8
FDT_WG_STAGES=4 run b1024_wg4 --steps 30 --warmup 8
run b1024_base2 --steps 30 --warmup 8
run b128_base --steps 40 --warmup 5 --global-batch 128
FDT_WG_FUSED_REDUCE=1 run b128_wgfr --steps 40 --warmup 5 --global-batch 128
FDT_WG_STAGES=4 run b128_wg4 --steps 40 --warmup 5 --global-batch 128
FDT_KGROUPS=0 run b128_kg0 --steps 40 --warmup 5 --global-batch 128
run b128_base2 --steps 40 --warmup 5 --global-batch 128
echo done
