#!/usr/bin/env bash
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r2i}
mkdir -p "$OUT"
timeout -k 10 500 python -u -m pytest tests/test_distributed_gpu.py tests/test_resnet_engine.py tests/test_transformer_graphs.py -m gpu -v -p no:cacheprovider --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1; rc=$?; echo "pytest rc=$rc" >> "$OUT/pytest.log"
case $rc in 0|1) ;; *) echo "pytest aborted rc=$rc"; exit 1;; esac
timeout -k 10 300 python bench.py --steps 30 --warmup 5 --global-batch 128 > "$OUT/bench128.log" 2>&1 || { echo bench128 failed; exit 1; }
timeout -k 10 300 python bench.py --model transformer --steps 20 --warmup 12 > "$OUT/bench_tr.log" 2>&1 || { echo bench_tr failed; exit 1; }
echo done
