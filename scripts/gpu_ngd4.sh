#!/usr/bin/env bash
# NGD fused W update: kernel + optimizer tests, step times, ResNet NGD+meta bench.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${1:-ngd4}
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_kernels.py -k "ngd" tests/test_ngd_graphs.py > "$OUT/pytest.log" 2>&1 || { echo pytest failed; tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
timeout -k 10 200 python scripts/bench_ngd.py --model resnet50 > "$OUT/bench_ngd.log" 2>&1 || exit 1
timeout -k 10 200 python scripts/bench_ngd.py --model transformer >> "$OUT/bench_ngd.log" 2>&1 || exit 1
cat "$OUT/bench_ngd.log" | grep -v amdgpu.ids
timeout -k 10 300 python bench.py --ngd --meta_learning --steps 20 --warmup 12 > "$OUT/ngd_meta.log" 2>&1 || exit 1
echo "ngd_meta $(grep -o '"ms_per_step": [0-9.]*' "$OUT/ngd_meta.log")"
