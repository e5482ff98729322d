#!/usr/bin/env bash
# Round 5: write-through conv epilogue stores A/B (+ engine numerics with them on).
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r5j}
mkdir -p "$OUT"
FDT_NATIVE=1 timeout -k 10 120 python -c "from faster_distributed_training_amd.ops import _native; _native.native()" || { echo "native extension stale or missing"; exit 1; }
FDT_CONV_WT=1 timeout -k 10 600 python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread \
  tests/test_resnet_engine.py tests/test_conv_kernels.py > "$OUT/pytest.log" 2>&1 || { echo tests failed; tail -20 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
run() {
  local name=$1; shift
  timeout -k 10 300 env "$@" > "$OUT/$name.log" 2>&1 || { echo "$name failed"; tail -5 "$OUT/$name.log"; exit 1; }
  grep -h '"value"' "$OUT/$name.log" > "$OUT/$name.json"
  echo "$name $(grep -o '"ms_per_step": [0-9.]*' "$OUT/$name.json")"
}
for i in 1 2; do
run bs1024_wt$i FDT_CONV_WT=1 python bench.py --steps 30 --warmup 8
run bs1024_plain$i FDT_CONV_WT=0 python bench.py --steps 30 --warmup 8
run bs128_wt$i FDT_CONV_WT=1 python bench.py --steps 40 --warmup 5 --global-batch 128
run bs128_plain$i FDT_CONV_WT=0 python bench.py --steps 40 --warmup 5 --global-batch 128
done
echo done
