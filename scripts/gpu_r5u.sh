#!/usr/bin/env bash
# Weight-gradient side branch: engine / deterministic / distributed / NGD GPU tests, A/B at both batches.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r5u}
mkdir -p "$OUT"
FDT_NATIVE=1 timeout -k 10 120 python -c "from faster_distributed_training_amd.ops import _native; _native.native()" || { echo "native extension stale or missing"; exit 1; }
timeout -k 10 900 python -u -m pytest tests/test_distributed_gpu.py tests/test_gpu_kernels.py -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1 ; rc=$?; echo "pytest rc=$rc"; grep -E "^(FAILED|ERROR)|AssertionError" "$OUT/pytest.log" | head -20; case $rc in 0|1) ;; *) exit 1;; esac
tail -1 "$OUT/pytest.log"
run() {
  local name=$1; shift
  timeout -k 10 300 python bench.py "$@" > "$OUT/$name.log" 2>&1 || { echo "$name failed"; tail -5 "$OUT/$name.log"; exit 1; }
  grep -h '"value"' "$OUT/$name.log" > "$OUT/$name.json"
  echo "$name $(grep -o '"ms_per_step": [0-9.]*' "$OUT/$name.json") $(grep -o '"graph_comm": "[^"]*"' "$OUT/$name.json")"
}
for rep in a b; do
FDT_WGRAD_BRANCH=0 run bs128_nobr_$rep --steps 40 --warmup 5 --global-batch 128
FDT_WGRAD_BRANCH=1 run bs128_br_$rep --steps 40 --warmup 5 --global-batch 128
done
FDT_WGRAD_BRANCH=0 run bs1024_nobr --steps 30 --warmup 8
FDT_WGRAD_BRANCH=1 run bs1024_br --steps 30 --warmup 8
FDT_WGRAD_BRANCH=1 run bs128_ddp_br --steps 40 --warmup 5 --global-batch 128 --ddp
echo done
