#!/usr/bin/env bash
# Session baseline (round 3, 2nd session): default bench, bs128, transformer B=256 / B=32,
# and a transformer kernel profile.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r3s2}
mkdir -p "$OUT"
run() {  # name, args...
  local name=$1; shift
  timeout -k 10 300 python bench.py "$@" > "$OUT/$name.log" 2>&1 || { echo "$name failed"; tail -5 "$OUT/$name.log"; exit 1; }
  grep -h '"value"' "$OUT/$name.log" > "$OUT/$name.json"
  echo "$name $(grep -o '"ms_per_step": [0-9.]*' "$OUT/$name.json")"
}
run bs1024 --steps 20 --warmup 5
run bs128 --steps 30 --warmup 5 --global-batch 128
run tr --model transformer --steps 20 --warmup 12
run tr32 --model transformer --global-batch 32 --steps 40 --warmup 12
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_tr" -o run -- python bench.py --model transformer --steps 10 --warmup 6 > "$OUT/prof_tr.log" 2>&1 || { echo prof failed; tail -20 "$OUT/prof_tr.log"; exit 1; }
f=$(find "$OUT/prof_tr" -name '*kernel_stats.csv' | head -n 1)
python scripts/kstats.py "$f" --steps 16 --top 60 > "$OUT/kstats_tr.txt"
echo done
