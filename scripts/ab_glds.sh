#!/usr/bin/env bash
# A/B of LDS-DMA staging (FDT_GLDS) for the prologue-free conv kernels: numerics, per-shape
# microbench and the 1-GPU bench, both settings in one call on one box.
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/glds
mkdir -p "$OUT"
FDT_GLDS=1 timeout -k 10 300 python -u -m pytest tests/test_conv_kernels.py tests/test_resnet_engine.py -x -q \
  -p no:cacheprovider --timeout 120 --timeout-method thread > "$OUT/t.log" 2>&1 || { tail -30 "$OUT/t.log"; exit 1; }
tail -2 "$OUT/t.log"
FDT_GLDS=1 timeout -k 10 200 python scripts/bench_conv.py --batch 1024 > "$OUT/bc_on.log" 2>&1 || exit 1
FDT_GLDS=0 timeout -k 10 200 python scripts/bench_conv.py --batch 1024 > "$OUT/bc_off.log" 2>&1 || exit 1
FDT_GLDS=1 timeout -k 10 200 python bench.py --steps 20 --warmup 5 > "$OUT/b_on.log" 2>&1 || exit 1
FDT_GLDS=0 timeout -k 10 200 python bench.py --steps 20 --warmup 5 > "$OUT/b_off.log" 2>&1 || exit 1
for f in "$OUT"/b_on.log "$OUT"/b_off.log; do grep -o '"ms_per_step": [0-9.]*' "$f"; done
tail -1 "$OUT/bc_on.log"
tail -1 "$OUT/bc_off.log"
