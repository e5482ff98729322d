#!/usr/bin/env bash
# K groups: conv numerics, re-tune batch 128 with kg in {1,2}, A/B the bench (old / new table).
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${1:-kg}
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_conv_kernels.py > "$OUT/pytest.log" 2>&1 || { echo pytest failed; tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
timeout -k 10 300 python bench.py --steps 30 --warmup 5 --global-batch 128 > "$OUT/bench128_old.log" 2>&1 || { tail "$OUT/bench128_old.log"; exit 1; }
timeout -k 10 900 python -u scripts/tune_conv.py --batches 128 --out "$OUT/tuned.json" > "$OUT/tune.log" 2>&1 || { echo tune failed; tail -5 "$OUT/tune.log"; exit 1; }
tail -2 "$OUT/tune.log"
cp "$OUT/tuned.json" faster_distributed_training_amd/ops/conv_tuned.json
timeout -k 10 300 python bench.py --steps 30 --warmup 5 --global-batch 128 > "$OUT/bench128_new.log" 2>&1 || { tail "$OUT/bench128_new.log"; exit 1; }
FDT_KGROUPS=0 timeout -k 10 300 python bench.py --steps 30 --warmup 5 --global-batch 128 > "$OUT/bench128_new_nokg.log" 2>&1 || exit 1
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > "$OUT/bench1024_new.log" 2>&1 || exit 1
for f in "$OUT"/bench*.log; do echo "$(basename $f) $(grep -o '"ms_per_step": [0-9.]*' $f)"; done
