#!/usr/bin/env bash
# RCCL event cache off: the distributed GPU tests + DDP benches.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r5al}
mkdir -p "$OUT"
FDT_NATIVE=1 timeout -k 10 120 python -c "from faster_distributed_training_amd.ops import _native; _native.native()" || { echo "native extension stale or missing"; exit 1; }
timeout -k 10 900 python -u -m pytest tests/test_distributed_gpu.py -m gpu -v -p no:cacheprovider --timeout 400 --timeout-method thread > "$OUT/pytest.log" 2>&1; rc=$?
echo "pytest rc=$rc"; tail -1 "$OUT/pytest.log"; grep -E "^(FAILED|ERROR)" "$OUT/pytest.log" | head
[ $rc -eq 0 ] || exit 1
run() {
  local name=$1; shift
  timeout -k 10 300 python bench.py "$@" > "$OUT/$name.log" 2>&1 || { echo "$name failed"; tail -5 "$OUT/$name.log"; exit 1; }
  grep -h '"value"' "$OUT/$name.log" > "$OUT/$name.json"
  echo "$name $(grep -o '"ms_per_step": [0-9.]*' "$OUT/$name.json") $(grep -o '"graph_comm": "[^"]*"' "$OUT/$name.json")"
}
run bs128 --steps 40 --warmup 5 --global-batch 128
run bs128_ddp --steps 40 --warmup 5 --global-batch 128 --ddp
run bs1024_ddp --steps 30 --warmup 8 --ddp
echo done
