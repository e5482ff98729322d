#!/usr/bin/env bash
# Deterministic-mode numerics, pinned staging tests, distributed GPU tests, memory-copy trace
# of the transformer bench (staged H2D on the copy stream, no pageable copies).
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r2e}
mkdir -p "$OUT"
timeout -k 10 300 python scripts/det_diag.py > "$OUT/det_diag.log" 2>&1 || { echo det_diag failed; exit 1; }
timeout -k 10 600 python -u -m pytest tests/test_prefetch.py tests/test_deterministic.py tests/test_distributed_gpu.py tests/test_resnet_engine.py -m gpu -v -p no:cacheprovider --timeout 200 --timeout-method thread > "$OUT/pytest.log" 2>&1; rc=$?; echo "pytest rc=$rc" >> "$OUT/pytest.log"
case $rc in 0|1) ;; *) echo "pytest aborted rc=$rc"; exit 1;; esac
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d "$OUT/copytrace" -o run -- python3 bench.py --model transformer --steps 10 --warmup 5 > "$OUT/copytrace.log" 2>&1 || { echo copytrace failed; exit 1; }
echo done
