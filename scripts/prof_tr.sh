#!/usr/bin/env bash
# Kernel-trace profile of the transformer bench (bs 256, L 128, NGD): 10 profiled steps.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${1:-prof_tr}
mkdir -p "$OUT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- python bench.py --model transformer --steps 10 --warmup 6 > "$OUT/prof.log" 2>&1 || { echo prof failed; tail -20 "$OUT/prof.log"; exit 1; }
f=$(find "$OUT/prof" -name '*kernel_stats.csv' | head -n 1)
python scripts/kstats.py "$f" --steps 16 --top 40 > "$OUT/kstats.txt"
cat "$OUT/kstats.txt"
