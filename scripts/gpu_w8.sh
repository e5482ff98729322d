#!/usr/bin/env bash
# Simulated 8-rank ZeRO-2 NGD: per-rank optimizer step time, cost- vs element-balanced split.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${1:-w8}
mkdir -p "$OUT"
timeout -k 10 300 python scripts/bench_ngd.py --model resnet50 --steps 32 --world 8 --balance ngd > "$OUT/bench_ngd_w8.log" 2>&1 || { tail "$OUT/bench_ngd_w8.log"; exit 1; }
timeout -k 10 300 python scripts/bench_ngd.py --model resnet50 --steps 32 --world 8 --balance numel >> "$OUT/bench_ngd_w8.log" 2>&1 || { tail "$OUT/bench_ngd_w8.log"; exit 1; }
timeout -k 10 300 python scripts/bench_ngd.py --model transformer --steps 32 --world 8 --balance ngd >> "$OUT/bench_ngd_w8.log" 2>&1 || { tail "$OUT/bench_ngd_w8.log"; exit 1; }
grep slowest "$OUT/bench_ngd_w8.log"
