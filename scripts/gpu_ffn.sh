#!/usr/bin/env bash
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${1:-ffn}
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_transformer_fusions.py tests/test_fused_epilogues.py > "$OUT/pytest.log" 2>&1 || { echo pytest failed; tail -40 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
timeout -k 10 300 python scripts/bench_ffn.py > "$OUT/bench_ffn.txt" 2>&1 || { tail "$OUT/bench_ffn.txt"; exit 1; }
cat "$OUT/bench_ffn.txt"
for v in 0 1; do
  FDT_FFN_FUSED=$v timeout -k 10 300 python bench.py --model transformer --steps 20 --warmup 12 > "$OUT/tr_$v.log" 2>&1 || { tail -5 "$OUT/tr_$v.log"; exit 1; }
  echo "tr fused=$v $(grep -o '"ms_per_step": [0-9.]*' "$OUT/tr_$v.log")"
done
