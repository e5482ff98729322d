#!/usr/bin/env bash
# DDP bucket size sweep on one GPU (world-1 RCCL group): cost of the graph cuts + actions.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${1:-ddp2}
mkdir -p "$OUT"
run() {
  local name=$1; shift
  timeout -k 10 300 python bench.py "$@" > "$OUT/$name.log" 2>&1 || { echo "$name failed"; tail -5 "$OUT/$name.log"; exit 1; }
  grep -h '"value"' "$OUT/$name.log" > "$OUT/$name.json"
  echo "$name $(grep -o '"ms_per_step": [0-9.]*' "$OUT/$name.json") $(grep -o '"ddp_buckets": [0-9]*' "$OUT/$name.json") $(grep -o '"bwd_graph_segments": [0-9]*' "$OUT/$name.json")"
}
run b128_plain --steps 40 --warmup 5 --global-batch 128
for mb in 16 25 50 100; do run b128_ddp$mb --steps 40 --warmup 5 --global-batch 128 --ddp --bucket-mb $mb; done
run b1024_plain --steps 20 --warmup 5
for mb in 25 50; do run b1024_ddp$mb --steps 20 --warmup 5 --ddp --bucket-mb $mb; done
