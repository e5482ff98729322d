#!/usr/bin/env bash
# Round 6: stride-2 3x3 data-gradient parity classes through the halo loop: numerics, per-layer
# timing, whole-step A/B.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r6ab}
mkdir -p "$OUT"
FDT_NATIVE=1 timeout -k 10 120 python -c "from faster_distributed_training_amd.ops import _native; _native.native()" || { echo "native extension stale or missing"; exit 1; }
timeout -k 10 300 python -u -m pytest tests/test_conv_kernels.py -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "h3" > "$OUT/pytest_h3.log" 2>&1; rc=$?
echo "pytest h3 rc=$rc"; tail -1 "$OUT/pytest_h3.log"
case $rc in 0) ;; 1) grep -E "^(FAILED|E )" "$OUT/pytest_h3.log" | head -20; exit 1;; *) echo aborted; tail -20 "$OUT/pytest_h3.log"; exit 1;; esac
for b in 1024 128; do
  timeout -k 10 300 python -u scripts/bench_s2.py --batch $b > "$OUT/bench_s2_$b.txt" 2>&1 || { echo "bench failed"; tail -10 "$OUT/bench_s2_$b.txt"; exit 1; }
  grep -v amdgpu.ids "$OUT/bench_s2_$b.txt"
done
j() { grep -h '"value"' "$OUT/$1.log" > "$OUT/$1.json"; echo "$1 $(grep -o '"ms_per_step": [0-9.]*' $OUT/$1.json)"; }
for v in 1 0 1 0; do
  FDT_CONV_H3_S2=$v timeout -k 10 300 python bench.py > "$OUT/bs1024_s2$v.log" 2>&1 || { echo "bench failed"; tail -5 "$OUT/bs1024_s2$v.log"; exit 1; }
  j bs1024_s2$v
done
