#!/usr/bin/env bash
# Round 5: the whole GPU test suite at HEAD (one process), smoke, headline bench, new bench rows.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r5l}
mkdir -p "$OUT"
FDT_NATIVE=1 timeout -k 10 120 python -c "from faster_distributed_training_amd.ops import _native; _native.native()" || { echo "native extension stale or missing"; exit 1; }
timeout -k 10 1500 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 400 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1; rc=$?
echo "pytest rc=$rc"; tail -1 "$OUT/pytest_gpu.log"
case $rc in 0) ;; 1) grep -E "^(FAILED|ERROR)" "$OUT/pytest_gpu.log" | head -20;; *) echo aborted; tail -20 "$OUT/pytest_gpu.log"; exit 1;; esac
grep -E "^\{'optimizer'" "$OUT/pytest_gpu.log" | cut -c1-600
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 && tail -1 "$OUT/smoke.log" || { echo smoke failed; tail -5 "$OUT/smoke.log"; exit 1; }
run() {
  local name=$1; shift
  timeout -k 10 300 python bench.py "$@" > "$OUT/$name.log" 2>&1 || { echo "$name failed"; tail -5 "$OUT/$name.log"; exit 1; }
  grep -h '"value"' "$OUT/$name.log" > "$OUT/$name.json"
  echo "$name $(grep -o '"ms_per_step": [0-9.]*' "$OUT/$name.json") $(grep -o '"graph_comm": "[^"]*"' "$OUT/$name.json")"
}
run bench_default
run tr_b256 --model transformer --steps 20 --warmup 12
run tr_b32 --model transformer --global-batch 32 --steps 40 --warmup 12
run tr_fsdp_offload --model transformer --fsdp --fsdp-offload --steps 10 --warmup 4
echo done
