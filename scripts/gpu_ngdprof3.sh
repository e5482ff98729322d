#!/usr/bin/env bash
# NGD optimizer step alone: timings + kernel profiles (ResNet-50 and transformer parameter sets).
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${1:-ngdprof3}
mkdir -p "$OUT"
timeout -k 10 200 python scripts/bench_ngd.py --model resnet50 > "$OUT/bench_ngd.log" 2>&1 || { echo bench_ngd failed; exit 1; }
timeout -k 10 200 python scripts/bench_ngd.py --model transformer >> "$OUT/bench_ngd.log" 2>&1 || { echo bench_ngd tr failed; exit 1; }
grep -v amdgpu.ids "$OUT/bench_ngd.log"
for m in resnet50 transformer; do
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_$m" -o run -- python3 scripts/bench_ngd.py --model $m --steps 48 > "$OUT/prof_$m.log" 2>&1 || { echo prof failed; exit 1; }
  f=$(find "$OUT/prof_$m" -name '*kernel_stats.csv' | head -n 1); python scripts/kstats.py "$f" --steps 48 --top 40 > "$OUT/kstats_$m.txt"
done
echo done
