#!/usr/bin/env bash
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r2m}
mkdir -p "$OUT"
timeout -k 10 120 ./tools/wg_rate > "$OUT/wg_rate.log" 2>&1 || { echo wg_rate failed; exit 1; }
timeout -k 10 300 python scripts/bench_membound.py --batch 1024 --reps 20 > "$OUT/membound.log" 2>&1 || { echo membound failed; exit 1; }
echo done
