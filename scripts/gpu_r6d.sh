#!/usr/bin/env bash
# Round 6: halo 3x3 loop with the conflict-free pixel map -- microbench, kernel + engine tests,
# whole-step bench (halo on / off), bs128.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r6d}
mkdir -p "$OUT"
FDT_NATIVE=1 timeout -k 10 120 python -c "from faster_distributed_training_amd.ops import _native; _native.native()" || { echo "native extension stale or missing"; exit 1; }
timeout -k 10 300 python -u scripts/bench_h3.py --batch 1024 > "$OUT/bench_h3_1024.txt" 2>&1 || { echo "bench_h3 failed"; tail -20 "$OUT/bench_h3_1024.txt"; exit 1; }
grep -v amdgpu.ids "$OUT/bench_h3_1024.txt"
timeout -k 10 600 python -u -m pytest tests/test_conv_kernels.py tests/test_resnet_engine.py -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > "$OUT/pytest.log" 2>&1; rc=$?
echo "pytest rc=$rc"; tail -1 "$OUT/pytest.log"
case $rc in 0) ;; 1) grep -E "^(FAILED|ERROR)|^E " "$OUT/pytest.log" | head -20; exit 1;; *) echo aborted; tail -20 "$OUT/pytest.log"; exit 1;; esac
for v in 1 0; do
  FDT_CONV_H3=$v timeout -k 10 300 python bench.py > "$OUT/bench_h3$v.log" 2>&1 || { echo "bench h3=$v failed"; tail -5 "$OUT/bench_h3$v.log"; exit 1; }
  grep -h '"value"' "$OUT/bench_h3$v.log" > "$OUT/bench_h3$v.json"; echo "bs1024 h3=$v $(grep -o '"ms_per_step": [0-9.]*' $OUT/bench_h3$v.json)"
  FDT_CONV_H3=$v timeout -k 10 300 python bench.py --global-batch 128 --steps 40 > "$OUT/bs128_h3$v.log" 2>&1 || { echo "bs128 h3=$v failed"; exit 1; }
  grep -h '"value"' "$OUT/bs128_h3$v.log" > "$OUT/bs128_h3$v.json"; echo "bs128 h3=$v $(grep -o '"ms_per_step": [0-9.]*' $OUT/bs128_h3$v.json)"
done
timeout -k 10 300 python -u scripts/bench_h3.py --batch 128 > "$OUT/bench_h3_128.txt" 2>&1 || { echo "bench_h3 128 failed"; exit 1; }
grep -v amdgpu.ids "$OUT/bench_h3_128.txt"
