#!/usr/bin/env bash
# Round 6: whole GPU suite on the current tree + bench A/B of the halo loop on one box.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r6i}
mkdir -p "$OUT"
FDT_NATIVE=1 timeout -k 10 120 python -c "from faster_distributed_training_amd.ops import _native; _native.native()" || { echo "native extension stale or missing"; exit 1; }
for v in 1 0 1; do
  FDT_CONV_H3=$v timeout -k 10 300 python bench.py > "$OUT/bench_h3$v.log" 2>&1 || { echo "bench h3=$v failed"; tail -5 "$OUT/bench_h3$v.log"; exit 1; }
  grep -h '"value"' "$OUT/bench_h3$v.log" >> "$OUT/bench_h3$v.json"; echo "bs1024 h3=$v $(grep -o '"ms_per_step": [0-9.]*' $OUT/bench_h3$v.log | tail -1)"
done
for v in 1 0; do
  FDT_CONV_H3=$v timeout -k 10 300 python bench.py --global-batch 128 --steps 40 > "$OUT/bs128_h3$v.log" 2>&1 || { echo "bs128 h3=$v failed"; exit 1; }
  grep -h '"value"' "$OUT/bs128_h3$v.log" > "$OUT/bs128_h3$v.json"; echo "bs128 h3=$v $(grep -o '"ms_per_step": [0-9.]*' $OUT/bs128_h3$v.json)"
done
timeout -k 10 1500 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 900 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1; rc=$?
echo "pytest rc=$rc"; tail -1 "$OUT/pytest_gpu.log"
case $rc in 0) ;; 1) grep -E "^(FAILED|ERROR)" "$OUT/pytest_gpu.log" | head -20;; *) echo aborted; tail -20 "$OUT/pytest_gpu.log"; exit 1;; esac
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 && tail -1 "$OUT/smoke.log" || { echo smoke failed; tail -5 "$OUT/smoke.log"; exit 1; }
