#!/usr/bin/env bash
# Final tree: whole GPU suite + smoke + the default bench and the 8-GPU-share bench.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r5am}
mkdir -p "$OUT"
FDT_NATIVE=1 timeout -k 10 120 python -c "from faster_distributed_training_amd.ops import _native; _native.native()" || { echo "native extension stale or missing"; exit 1; }
timeout -k 10 1500 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 400 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1; rc=$?
echo "pytest rc=$rc"; tail -1 "$OUT/pytest_gpu.log"
case $rc in 0) ;; 1) grep -E "^(FAILED|ERROR)" "$OUT/pytest_gpu.log" | head -20;; *) echo aborted; tail -20 "$OUT/pytest_gpu.log"; exit 1;; esac
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 && tail -1 "$OUT/smoke.log" || { echo smoke failed; tail -5 "$OUT/smoke.log"; exit 1; }
timeout -k 10 300 python bench.py > "$OUT/bench_default.log" 2>&1 || { echo "bench failed"; tail -5 "$OUT/bench_default.log"; exit 1; }
grep -h '"value"' "$OUT/bench_default.log" > "$OUT/bench_default.json"; grep -o '"ms_per_step": [0-9.]*' "$OUT/bench_default.json"
timeout -k 10 300 python bench.py --steps 40 --warmup 5 --global-batch 128 > "$OUT/bs128.log" 2>&1 || { echo "bs128 failed"; exit 1; }
grep -h '"value"' "$OUT/bs128.log" > "$OUT/bs128.json"; grep -o '"ms_per_step": [0-9.]*' "$OUT/bs128.json"
echo done
