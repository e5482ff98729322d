#!/usr/bin/env bash
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${1:-det}
mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_optim.py -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1; tail -4 "$OUT/pytest.log"; grep -B3 -A6 "^E " "$OUT/pytest.log" | head -30
timeout -k 10 200 python scripts/bench_ngd.py --model resnet50 --steps 40 > "$OUT/bench_ngd.log" 2>&1 || { tail "$OUT/bench_ngd.log"; exit 1; }
timeout -k 10 200 python scripts/bench_ngd.py --model transformer --steps 40 >> "$OUT/bench_ngd.log" 2>&1 || { tail "$OUT/bench_ngd.log"; exit 1; }
grep steps "$OUT/bench_ngd.log"
