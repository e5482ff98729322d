#!/usr/bin/env bash
# The multi-GPU data-parallel path on one GPU: DDP bucket reducer over a world-1 RCCL group
# (graph segments cut at every bucket, all-reduce actions between them) vs plain, bs128 / bs1024.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${1:-ddp1}
mkdir -p "$OUT"
run() {
  local name=$1; shift
  timeout -k 10 300 python bench.py "$@" > "$OUT/$name.log" 2>&1 || { echo "$name failed"; tail -5 "$OUT/$name.log"; exit 1; }
  grep -h '"value"' "$OUT/$name.log" > "$OUT/$name.json"
  echo "$name $(grep -o '"ms_per_step": [0-9.]*' "$OUT/$name.json") $(grep -o '"ddp_buckets": [0-9]*' "$OUT/$name.json") $(grep -o '"bwd_graph_segments": [0-9]*' "$OUT/$name.json")"
}
run b128_plain --steps 40 --warmup 5 --global-batch 128
run b128_ddp --steps 40 --warmup 5 --global-batch 128 --ddp
run b128_ddp25 --steps 40 --warmup 5 --global-batch 128 --ddp --bucket-mb 25
run b1024_ddp --steps 20 --warmup 5 --ddp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/prof128" -o run -- python3 bench.py --steps 4 --warmup 3 --global-batch 128 --ddp > "$OUT/prof128.log" 2>&1 || { echo prof failed; tail "$OUT/prof128.log"; exit 1; }
f=$(find "$OUT/prof128" -name '*kernel_trace.csv' | head -n 1)
python scripts/ktrace_step.py "$f" > "$OUT/timeline128_ddp.txt"
head -1 "$OUT/timeline128_ddp.txt"
