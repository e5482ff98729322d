#!/usr/bin/env bash
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r2o}
mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest tests/test_conv_kernels.py tests/test_resnet_engine.py -m gpu -q -p no:cacheprovider --timeout 200 --timeout-method thread > "$OUT/pytest.log" 2>&1; rc=$?; echo "pytest rc=$rc" >> "$OUT/pytest.log"
case $rc in 0) ;; *) echo "pytest failed rc=$rc"; exit 1;; esac
timeout -k 10 400 python scripts/bench_membound.py --batch 1024 --reps 20 --tile 128,128,32 --ops fwd,store,add,actb,join > "$OUT/membound.log" 2>&1 || { echo membound failed; exit 1; }
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > "$OUT/bench.log" 2>&1 || { echo bench failed; exit 1; }
timeout -k 10 300 python bench.py --steps 30 --warmup 5 --global-batch 128 > "$OUT/bench128.log" 2>&1 || { echo bench128 failed; exit 1; }
echo done
