#!/usr/bin/env bash
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${1:-ffn2}
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_transformer_fusions.py > "$OUT/pytest.log" 2>&1 || { echo pytest failed; tail -40 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
for spec in "0 both" "1 both" "1 bwd" "1 fwd" "0 both" "1 both"; do
  set -- $spec
  FDT_FFN_FUSED=$1 FDT_FFN_FUSED_SIDES=$2 timeout -k 10 300 python bench.py --model transformer --steps 30 --warmup 12 > "$OUT/tr_$1_$2.log" 2>&1 || { tail -5 "$OUT/tr_$1_$2.log"; exit 1; }
  echo "tr fused=$1 sides=$2 $(grep -o '"ms_per_step": [0-9.]*' "$OUT/tr_$1_$2.log")"
done
