#!/usr/bin/env bash
# Re-tune the batch-1024 fwd/dgrad table with K groups, then A/B the bench.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${1:-tune1024kg}
mkdir -p "$OUT"
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > "$OUT/bench1024_old.log" 2>&1 || exit 1
timeout -k 10 1000 python -u scripts/tune_conv.py --batches 1024 --ops fwd,dgrad --splits 1 2 4 --out "$OUT/tuned.json" > "$OUT/tune.log" 2>&1 || { echo tune failed; tail -5 "$OUT/tune.log"; exit 1; }
tail -2 "$OUT/tune.log"
cp "$OUT/tuned.json" faster_distributed_training_amd/ops/conv_tuned.json
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > "$OUT/bench1024_new.log" 2>&1 || exit 1
FDT_KGROUPS=0 timeout -k 10 300 python bench.py --steps 20 --warmup 5 > "$OUT/bench1024_new_nokg.log" 2>&1 || exit 1
timeout -k 10 300 python bench.py --steps 30 --warmup 5 --global-batch 128 > "$OUT/bench128_new.log" 2>&1 || exit 1
for f in "$OUT"/bench*.log; do echo "$(basename $f) $(grep -o '"ms_per_step": [0-9.]*' $f)"; done
