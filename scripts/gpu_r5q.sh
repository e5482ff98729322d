#!/usr/bin/env bash
# Join fold widened to 128 / 256-channel next convs: kernel + engine tests, A/B at both batches.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r5q}
mkdir -p "$OUT"
FDT_NATIVE=1 timeout -k 10 120 python -c "from faster_distributed_training_amd.ops import _native; _native.native()" || { echo "native extension stale or missing"; exit 1; }
timeout -k 10 600 python -u -m pytest tests/test_conv_kernels.py tests/test_resnet_engine.py tests/test_deterministic.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { echo "pytest failed"; tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
run() {
  local name=$1; shift
  timeout -k 10 300 python bench.py "$@" > "$OUT/$name.log" 2>&1 || { echo "$name failed"; tail -5 "$OUT/$name.log"; exit 1; }
  grep -h '"value"' "$OUT/$name.log" > "$OUT/$name.json"
  echo "$name $(grep -o '"ms_per_step": [0-9.]*' "$OUT/$name.json")"
}
for rep in a b; do
FDT_JOIN_FOLD_MIN_M=262144 FDT_EW_UNROLL=0 run bs128_none_ew0_$rep --steps 40 --warmup 5 --global-batch 128
FDT_JOIN_FOLD_MIN_M=262144 FDT_EW_UNROLL=1 run bs128_none_ew1_$rep --steps 40 --warmup 5 --global-batch 128
FDT_JOIN_FOLD_MIN_M=65536 FDT_EW_UNROLL=1 run bs128_m16_$rep --steps 40 --warmup 5 --global-batch 128
FDT_JOIN_FOLD_MIN_M=32768 FDT_EW_UNROLL=1 run bs128_m15_$rep --steps 40 --warmup 5 --global-batch 128
done
run bs1024_default --steps 30 --warmup 8
echo done
