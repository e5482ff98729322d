#!/usr/bin/env bash
# Round 4: kernel-trace of ResNet-50 bs128 plain vs the DDP reducer path at world 1.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r4p}
mkdir -p "$OUT"
prof() {
  local name=$1 steps=$2; shift 2
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/$name" -o run -- python bench.py "$@" > "$OUT/$name.log" 2>&1 || { echo "$name failed"; tail -20 "$OUT/$name.log"; exit 1; }
  f=$(find "$OUT/$name" -name '*kernel_stats.csv' | head -n 1)
  python scripts/kstats.py "$f" --steps "$steps" --top 80 > "$OUT/kstats_$name.txt"
  head -1 "$OUT/kstats_$name.txt"; grep -h '"value"' "$OUT/$name.log" | grep -o '"ms_per_step": [0-9.]*'
}
prof plain 35 --global-batch 128 --steps 30 --warmup 5
prof ddp 35 --global-batch 128 --steps 30 --warmup 5 --ddp
echo done
