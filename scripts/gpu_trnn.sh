#!/usr/bin/env bash
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${1:-trnn}
mkdir -p "$OUT"
timeout -k 10 300 python bench.py --model transformer --no-native --steps 10 --warmup 12 > "$OUT/tr_nonative.log" 2>&1 || { echo tr_nonative failed; grep -v "^frame" "$OUT/tr_nonative.log" | tail -8; exit 1; }
grep -h '"value"' "$OUT/tr_nonative.log" | cut -c1-200
timeout -k 10 300 python -u -m pytest tests/test_transformer_graphs.py tests/test_transformer_fusions.py -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1; tail -1 "$OUT/pytest.log"
