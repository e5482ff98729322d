#!/usr/bin/env bash
# NGD GPU check: kernel/numerics tests, the optimizer-step microbench on the real ResNet-50
# parameter set, and the ResNet-50 bs1024 --ngd --meta_learning bench (one JSON line).
#   bash scripts/gpu_ngd.sh [OUT]
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${1:-ngd}
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k ngd \
  -p no:cacheprovider > "$OUT/t.log" 2>&1 || { tail -40 "$OUT/t.log"; exit 1; }
tail -1 "$OUT/t.log"
timeout -k 10 200 python scripts/bench_ngd.py --model resnet50 --steps 24 2>&1 | tee "$OUT/ngd_step.log" || exit 1
timeout -k 10 200 python scripts/bench_ngd.py --model transformer --steps 24 2>&1 | tee -a "$OUT/ngd_step.log" || exit 1
timeout -k 10 300 python bench.py --ngd --meta_learning --steps 20 --warmup 12 > "$OUT/b.log" 2>&1 || { tail -5 "$OUT/b.log"; exit 1; }
grep -h '"value"' "$OUT/b.log" | tee "$OUT/ngd_meta.json"
