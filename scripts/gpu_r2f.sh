#!/usr/bin/env bash
# BK=128 conv tiles + fence-free split-K: conv kernel tests, engine tests, small-M retune at
# batch 128 (into a scratch table), benches with the in-tree table.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r2f}
mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest tests/test_conv_kernels.py tests/test_resnet_engine.py tests/test_deterministic.py -m gpu -q -p no:cacheprovider --timeout 200 --timeout-method thread > "$OUT/pytest.log" 2>&1; rc=$?; echo "pytest rc=$rc" >> "$OUT/pytest.log"
case $rc in 0) ;; *) echo "pytest failed rc=$rc"; exit 1;; esac
timeout -k 10 300 python bench.py --steps 30 --warmup 5 --global-batch 128 > "$OUT/bench128_pre.log" 2>&1 || { echo bench128 failed; exit 1; }
timeout -k 10 900 python -u scripts/tune_conv.py --batches 128 --max-m 8192 --out "$OUT/tuned128.json" > "$OUT/tune.log" 2>&1 || { echo tune failed; exit 1; }
echo done
