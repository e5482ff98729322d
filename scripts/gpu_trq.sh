#!/usr/bin/env bash
# Quick transformer iteration: epilogue kernel tests, bench B=256, kernel stats.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${1:-trq}
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_fused_epilogues.py tests/test_transformer_fusions.py > "$OUT/pytest.log" 2>&1 || { echo pytest failed; tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
timeout -k 10 300 python bench.py --model transformer --steps 20 --warmup 12 > "$OUT/tr.log" 2>&1 || { echo tr failed; tail -5 "$OUT/tr.log"; exit 1; }
echo "tr $(grep -o '"ms_per_step": [0-9.]*' "$OUT/tr.log")"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_tr" -o run -- python bench.py --model transformer --steps 10 --warmup 6 > "$OUT/prof_tr.log" 2>&1 || { echo prof failed; tail -20 "$OUT/prof_tr.log"; exit 1; }
f=$(find "$OUT/prof_tr" -name '*kernel_stats.csv' | head -n 1)
python scripts/kstats.py "$f" --steps 16 --top 60 > "$OUT/kstats_tr.txt"
grep -E "colsum|dropout|gelu" "$OUT/kstats_tr.txt"
