#!/usr/bin/env bash
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${1:-side}
mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_optim.py tests/test_transformer_graphs.py -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1; tail -4 "$OUT/pytest.log"
timeout -k 10 300 python bench.py --model transformer --steps 20 --warmup 12 > "$OUT/bench_tr.log" 2>&1 || { tail "$OUT/bench_tr.log"; exit 1; }
grep '"value"' "$OUT/bench_tr.log" | cut -c1-200
timeout -k 10 300 python bench.py --ngd --meta_learning --steps 20 --warmup 15 > "$OUT/bench_ngd_meta.log" 2>&1 || { tail "$OUT/bench_ngd_meta.log"; exit 1; }
grep '"value"' "$OUT/bench_ngd_meta.log" | cut -c1-200
