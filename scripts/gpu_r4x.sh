#!/usr/bin/env bash
# Round 4: NGD eigensolve overlapped on a side stream (default) vs inline on the main stream.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r4x}
mkdir -p "$OUT"
run() {
  local name=$1; shift
  timeout -k 10 300 python bench.py "$@" > "$OUT/$name.log" 2>&1 || { echo "$name failed"; tail -5 "$OUT/$name.log"; exit 1; }
  grep -h '"value"' "$OUT/$name.log" > "$OUT/$name.json"
  echo "$name $(grep -o '"ms_per_step": [0-9.]*' "$OUT/$name.json")"
}
run tr_b32 --model transformer --global-batch 32 --steps 60 --warmup 12
FDT_NGD_OVERLAP=0 run tr_b32_inline --model transformer --global-batch 32 --steps 60 --warmup 12
run tr_b256 --model transformer --steps 24 --warmup 12
FDT_NGD_OVERLAP=0 run tr_b256_inline --model transformer --steps 24 --warmup 12
run ngd_meta --ngd --meta_learning --steps 24 --warmup 12
FDT_NGD_OVERLAP=0 run ngd_meta_inline --ngd --meta_learning --steps 24 --warmup 12
echo done
