#!/usr/bin/env bash
# Round 5 start: HEAD numbers at bs1024 / bs128 / bs128 --ddp plus per-kernel traces of one step.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r5a}
mkdir -p "$OUT"
run() {
  local name=$1; shift
  timeout -k 10 300 python bench.py "$@" > "$OUT/$name.log" 2>&1 || { echo "$name failed"; tail -5 "$OUT/$name.log"; exit 1; }
  grep -h '"value"' "$OUT/$name.log" > "$OUT/$name.json"
  echo "$name $(grep -o '"ms_per_step": [0-9.]*' "$OUT/$name.json") $(grep -o '"host_ms_per_step": [0-9.]*' "$OUT/$name.json")"
}
prof() {
  local name=$1 steps=$2; shift 2
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_$name" -o run -- python3 bench.py "$@" > "$OUT/prof_$name.log" 2>&1 || { echo "prof $name failed"; tail -5 "$OUT/prof_$name.log"; exit 1; }
  f=$(find "$OUT/prof_$name" -name '*kernel_stats.csv' | head -n 1)
  python scripts/kstats.py "$f" --steps "$steps" --top 60 > "$OUT/kstats_$name.txt"
  head -3 "$OUT/kstats_$name.txt"
}
run bs1024 --steps 30 --warmup 8
run bs128 --steps 40 --warmup 5 --global-batch 128
run bs128_ddp --steps 40 --warmup 5 --global-batch 128 --ddp
prof bs128 15 --steps 10 --warmup 5 --global-batch 128
prof bs1024 7 --steps 4 --warmup 3
echo done
