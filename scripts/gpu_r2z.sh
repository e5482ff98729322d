#!/usr/bin/env bash
# NGD kernel tests, NGD step bench, transformer bench, ResNet NGD+meta bench.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r2z}
mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_optim.py -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
timeout -k 10 200 python scripts/bench_ngd.py --model resnet50 --steps 40 > "$OUT/bench_ngd.log" 2>&1 || { tail "$OUT/bench_ngd.log"; exit 1; }
timeout -k 10 200 python scripts/bench_ngd.py --model transformer --steps 40 >> "$OUT/bench_ngd.log" 2>&1 || { tail "$OUT/bench_ngd.log"; exit 1; }
grep steps "$OUT/bench_ngd.log"
timeout -k 10 300 python bench.py --model transformer --steps 20 --warmup 12 > "$OUT/bench_tr.log" 2>&1 || { tail "$OUT/bench_tr.log"; exit 1; }
grep '"value"' "$OUT/bench_tr.log" | cut -c1-200
timeout -k 10 300 python bench.py --ngd --meta_learning --steps 20 --warmup 15 > "$OUT/bench_ngd_meta.log" 2>&1 || { tail "$OUT/bench_ngd_meta.log"; exit 1; }
grep '"value"' "$OUT/bench_ngd_meta.log" | cut -c1-200
timeout -k 10 300 python scripts/bench_ngd.py --model resnet50 --steps 32 --world 8 --balance ngd > "$OUT/bench_ngd_w8.log" 2>&1 && timeout -k 10 300 python scripts/bench_ngd.py --model resnet50 --steps 32 --world 8 --balance numel >> "$OUT/bench_ngd_w8.log" 2>&1 || { tail "$OUT/bench_ngd_w8.log"; exit 1; }
grep world "$OUT/bench_ngd_w8.log"
