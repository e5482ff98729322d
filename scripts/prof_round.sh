#!/usr/bin/env bash
# Kernel-trace profile of the bench at a given per-GPU batch + per-shape conv microbench.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${1:-prof}
GB=${2:-128}
mkdir -p "$OUT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof$GB" -o run -- python bench.py --steps 4 --warmup 3 --global-batch $GB > "$OUT/prof$GB.log" 2>&1 || { echo prof failed; exit 1; }
timeout -k 10 300 python scripts/bench_conv.py --batch 1024 > "$OUT/bench_conv1024.log" 2>&1 || { echo bench_conv failed; exit 1; }
timeout -k 10 300 python scripts/bench_conv.py --batch 128 > "$OUT/bench_conv128.log" 2>&1 || { echo bench_conv failed; exit 1; }
echo done
