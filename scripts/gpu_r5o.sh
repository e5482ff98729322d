#!/usr/bin/env bash
# Wide slot rows for large-M 3x3 statistics producers: A/B at batch 1024 + a kernel profile.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r5o}
mkdir -p "$OUT"
FDT_NATIVE=1 timeout -k 10 120 python -c "from faster_distributed_training_amd.ops import _native; _native.native()" || { echo "native extension stale or missing"; exit 1; }
run() {
  local name=$1; shift
  timeout -k 10 300 python bench.py "$@" > "$OUT/$name.log" 2>&1 || { echo "$name failed"; tail -5 "$OUT/$name.log"; exit 1; }
  grep -h '"value"' "$OUT/$name.log" > "$OUT/$name.json"
  echo "$name $(grep -o '"ms_per_step": [0-9.]*' "$OUT/$name.json")"
}
FDT_STAT_WIDE_ROWS=0 run bs1024_w0a --steps 30 --warmup 8
FDT_STAT_WIDE_ROWS=256 run bs1024_w256a --steps 30 --warmup 8
FDT_STAT_WIDE_ROWS=0 run bs1024_w0b --steps 30 --warmup 8
FDT_STAT_WIDE_ROWS=256 run bs1024_w256b --steps 30 --warmup 8
FDT_STAT_WIDE_ROWS=1024 run bs1024_w1024 --steps 30 --warmup 8
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_bs1024" -o run -- python3 bench.py --steps 4 --warmup 3 > "$OUT/prof_bs1024.log" 2>&1 || { echo "prof failed"; tail -5 "$OUT/prof_bs1024.log"; exit 1; }
f=$(find "$OUT/prof_bs1024" -name '*kernel_stats.csv' | head -n 1)
python scripts/kstats.py "$f" --steps 7 --top 80 > "$OUT/kstats_bs1024.txt"
head -3 "$OUT/kstats_bs1024.txt"
echo done
