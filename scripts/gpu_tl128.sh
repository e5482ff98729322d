#!/usr/bin/env bash
# Kernel-trace timeline of one graph-replayed ResNet-50 step at batch 128 and 1024.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${1:-tl128}
mkdir -p "$OUT"
for gb in 128 1024; do
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/prof$gb" -o run -- python3 bench.py --steps 4 --warmup 3 --global-batch $gb > "$OUT/prof$gb.log" 2>&1 || { echo prof failed; tail "$OUT/prof$gb.log"; exit 1; }
  f=$(find "$OUT/prof$gb" -name '*kernel_trace.csv' | head -n 1)
  python scripts/ktrace_step.py "$f" > "$OUT/timeline$gb.txt"
  head -1 "$OUT/timeline$gb.txt"
done
