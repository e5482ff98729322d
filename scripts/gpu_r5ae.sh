#!/usr/bin/env bash
# NGD clip scale deferred to the SGD kernel on plain steps: NGD GPU tests + transformer benches.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r5ae}
mkdir -p "$OUT"
FDT_NATIVE=1 timeout -k 10 120 python -c "from faster_distributed_training_amd.ops import _native; _native.native()" || { echo "native extension stale or missing"; exit 1; }
timeout -k 10 900 python -u -m pytest tests/test_ngd_graphs.py tests/test_gpu_kernels.py tests/test_distributed_gpu.py -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread -k "ngd or sharded or transformer" > "$OUT/pytest.log" 2>&1; rc=$?
echo "pytest rc=$rc"; tail -1 "$OUT/pytest.log"; grep -E "^(FAILED|ERROR)" "$OUT/pytest.log" | head; case $rc in 0|1) ;; *) exit 1;; esac
run() {
  local name=$1; shift
  timeout -k 10 300 python bench.py "$@" > "$OUT/$name.log" 2>&1 || { echo "$name failed"; tail -5 "$OUT/$name.log"; exit 1; }
  grep -h '"value"' "$OUT/$name.log" > "$OUT/$name.json"
  echo "$name $(grep -o '"ms_per_step": [0-9.]*' "$OUT/$name.json")"
}
FDT_NGD_DEFER_SCALE=0 run tr_b32_nodefer --model transformer --global-batch 32 --steps 40 --warmup 12
run tr_b32_a --model transformer --global-batch 32 --steps 40 --warmup 12
FDT_NGD_DEFER_SCALE=0 run tr_b32_nodefer_b --model transformer --global-batch 32 --steps 40 --warmup 12
run tr_b32_b --model transformer --global-batch 32 --steps 40 --warmup 12
run tr_b256 --model transformer --steps 20 --warmup 12
run bs128 --steps 40 --warmup 5 --global-batch 128
run bs1024 --steps 30 --warmup 8
echo done
