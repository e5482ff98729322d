#!/usr/bin/env bash
# Round 6: final-tree check after the launch-table updates: engine tests + headline benches.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r6ag}
mkdir -p "$OUT"
FDT_NATIVE=1 timeout -k 10 120 python -c "from faster_distributed_training_amd.ops import _native; _native.native()" || { echo "native extension stale or missing"; exit 1; }
timeout -k 10 600 python -u -m pytest tests/test_resnet_engine.py tests/test_conv_kernels.py tests/test_deterministic.py -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread > "$OUT/pytest_engine.log" 2>&1; rc=$?
echo "pytest rc=$rc"; tail -1 "$OUT/pytest_engine.log"
case $rc in 0) ;; 1) grep -E "^(FAILED|ERROR)" "$OUT/pytest_engine.log" | head -20;; *) echo aborted; tail -20 "$OUT/pytest_engine.log"; exit 1;; esac
j() { grep -h '"value"' "$OUT/$1.log" > "$OUT/$1.json"; echo "$1 $(grep -o '"ms_per_step": [0-9.]*' $OUT/$1.json)"; }
timeout -k 10 300 python bench.py > "$OUT/bench_default.log" 2>&1 || { echo "bench failed"; tail -5 "$OUT/bench_default.log"; exit 1; }
j bench_default
timeout -k 10 300 python bench.py --global-batch 128 --steps 40 > "$OUT/bs128.log" 2>&1 || { echo "bs128 failed"; exit 1; }
j bs128
timeout -k 10 300 python bench.py > "$OUT/bench_default2.log" 2>&1 || { echo "bench failed"; exit 1; }
j bench_default2
