#!/usr/bin/env bash
# Transformer at the 8-GPU per-GPU share (B = 32): step time and GPU busy fraction (kernel trace).
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${1:-b32}
mkdir -p "$OUT"
timeout -k 10 300 python bench.py --model transformer --global-batch 32 --steps 40 --warmup 12 > "$OUT/bench_tr32.log" 2>&1 || { tail "$OUT/bench_tr32.log"; exit 1; }
grep '"value"' "$OUT/bench_tr32.log" | cut -c1-200
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/prof" -o run -- python3 bench.py --model transformer --global-batch 32 --steps 30 --warmup 12 > "$OUT/prof.log" 2>&1 || { echo prof failed; tail "$OUT/prof.log"; exit 1; }
f=$(find "$OUT/prof" -name '*kernel_trace.csv' | head -n 1)
python scripts/busy_fraction.py "$f" --marker sgd_kernel --steps 20 | tee "$OUT/busy.txt"
