#!/usr/bin/env bash
# Round 6: fragment-pipelined halo weight gradient: numerics, per-layer timing, whole step A/B.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r6r}
mkdir -p "$OUT"
FDT_NATIVE=1 timeout -k 10 120 python -c "from faster_distributed_training_amd.ops import _native; _native.native()" || { echo "native extension stale or missing"; exit 1; }
timeout -k 10 300 python -u -m pytest tests/test_conv_kernels.py -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "h3_conv_wgrad" > "$OUT/pytest_wh3.log" 2>&1; rc=$?
echo "pytest wh3 rc=$rc"; tail -1 "$OUT/pytest_wh3.log"
case $rc in 0) ;; 1) grep -E "^(FAILED|E )" "$OUT/pytest_wh3.log" | head -20; exit 1;; *) echo aborted; tail -20 "$OUT/pytest_wh3.log"; exit 1;; esac
timeout -k 10 300 python -u scripts/bench_h3.py --batch 1024 --only wgrad > "$OUT/bench_wh3_1024.txt" 2>&1 || { echo "bench failed"; tail -20 "$OUT/bench_wh3_1024.txt"; exit 1; }
grep -v amdgpu.ids "$OUT/bench_wh3_1024.txt"
j() { grep -h '"value"' "$OUT/$1.log" > "$OUT/$1.json"; echo "$1 $(grep -o '"ms_per_step": [0-9.]*' $OUT/$1.json)"; }
for v in 1 0 1 0; do
  FDT_WGRAD_H3=$v timeout -k 10 300 python bench.py > "$OUT/bs1024_wh3$v.log" 2>&1 || { echo "bench failed"; tail -5 "$OUT/bs1024_wh3$v.log"; exit 1; }
  j bs1024_wh3$v
done
