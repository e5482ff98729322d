#!/usr/bin/env bash
# Kernel-trace profile of the NGD optimizer step alone (ResNet-50 and transformer parameter sets).
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${1:-ngdprof}
mkdir -p "$OUT"
timeout -k 10 200 python scripts/bench_ngd.py --model resnet50 > "$OUT/bench_ngd.log" 2>&1 || { echo bench_ngd failed; exit 1; }
timeout -k 10 200 python scripts/bench_ngd.py --model transformer >> "$OUT/bench_ngd.log" 2>&1 || { echo bench_ngd tr failed; exit 1; }
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- python3 scripts/bench_ngd.py --model resnet50 --steps 10 > "$OUT/prof.log" 2>&1 || { echo prof failed; exit 1; }

f=$(find "$OUT/prof" -name '*kernel_stats.csv' | head -n 1)
python scripts/kstats.py "$f" --steps 10 --top 40 > "$OUT/kstats_ngd.txt"
cat "$OUT/bench_ngd.log"
