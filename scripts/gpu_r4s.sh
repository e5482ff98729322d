#!/usr/bin/env bash
# Round 4: transformer A/B at 32 samples: FFN GEMM epilogues, NGD graph replay.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r4s}
mkdir -p "$OUT"
run() {
  local name=$1; shift
  timeout -k 10 300 python bench.py "$@" > "$OUT/$name.log" 2>&1 || { echo "$name failed"; tail -5 "$OUT/$name.log"; exit 1; }
  grep -h '"value"' "$OUT/$name.log" > "$OUT/$name.json"
  echo "$name $(grep -o '"ms_per_step": [0-9.]*' "$OUT/$name.json") $(grep -o '"host_ms_per_step": [0-9.]*' "$OUT/$name.json")"
}
run tr_b32 --model transformer --global-batch 32 --steps 60 --warmup 12
FDT_FFN_FUSED=1 run tr_b32_ffn --model transformer --global-batch 32 --steps 60 --warmup 12
FDT_NGD_GRAPHS=1 run tr_b32_ngdg --model transformer --global-batch 32 --steps 60 --warmup 12
FDT_NGD_GRAPHS=1 run tr_b256_ngdg --model transformer --steps 20 --warmup 12
run tr_b256 --model transformer --steps 20 --warmup 12
FDT_FFN_FUSED=1 run tr_b256_ffn --model transformer --steps 20 --warmup 12
echo done
