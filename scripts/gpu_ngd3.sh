#!/usr/bin/env bash
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${1:-ngd3}
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread -k ngd > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
timeout -k 10 200 python scripts/bench_ngd.py --model resnet50 --steps 40 > "$OUT/bench_ngd.log" 2>&1 || { tail "$OUT/bench_ngd.log"; exit 1; }
timeout -k 10 200 python scripts/bench_ngd.py --model transformer --steps 40 >> "$OUT/bench_ngd.log" 2>&1 || { tail "$OUT/bench_ngd.log"; exit 1; }
grep steps "$OUT/bench_ngd.log"
timeout -k 10 300 python bench.py --model transformer --steps 20 --warmup 12 > "$OUT/bench_tr.log" 2>&1 || { tail "$OUT/bench_tr.log"; exit 1; }
grep '"value"' "$OUT/bench_tr.log" | cut -c1-200
bash scripts/pmc_ngd.sh "$(basename $OUT)_pmc" | grep "489472\|425984"
