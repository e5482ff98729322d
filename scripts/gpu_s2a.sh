#!/usr/bin/env bash
# GPU tests of this session's changes + transformer bench / profile.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${1:-s2a}
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_fused_epilogues.py tests/test_transformer_fusions.py tests/test_prefetch.py tests/test_transformer_graphs.py \
  tests/test_distributed_gpu.py > "$OUT/pytest.log" 2>&1 || { echo pytest failed; tail -30 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
for spec in "tr --model transformer --steps 20 --warmup 12" "tr32 --model transformer --global-batch 32 --steps 40 --warmup 12"; do
  set -- $spec; name=$1; shift
  timeout -k 10 300 python bench.py "$@" > "$OUT/$name.log" 2>&1 || { echo "$name failed"; tail -5 "$OUT/$name.log"; exit 1; }
  echo "$name $(grep -o '"ms_per_step": [0-9.]*' "$OUT/$name.log")"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_tr" -o run -- python bench.py --model transformer --steps 10 --warmup 6 > "$OUT/prof_tr.log" 2>&1 || { echo prof failed; tail -20 "$OUT/prof_tr.log"; exit 1; }
f=$(find "$OUT/prof_tr" -name '*kernel_stats.csv' | head -n 1)
python scripts/kstats.py "$f" --steps 16 --top 60 > "$OUT/kstats_tr.txt"
echo done
