#!/usr/bin/env bash
# Round 5: lazy-statistics scope A/B (none / elementwise / all), bs128 x3 and bs1024.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r5d}
mkdir -p "$OUT"
run() {
  local name=$1; shift
  timeout -k 10 300 env "$@" > "$OUT/$name.log" 2>&1 || { echo "$name failed"; tail -5 "$OUT/$name.log"; exit 1; }
  grep -h '"value"' "$OUT/$name.log" > "$OUT/$name.json"
  echo "$name $(grep -o '"ms_per_step": [0-9.]*' "$OUT/$name.json")"
}
timeout -k 10 600 python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread \
  tests/test_resnet_engine.py > "$OUT/pytest_engine.log" 2>&1 || { echo "engine tests failed"; tail -20 "$OUT/pytest_engine.log"; exit 1; }
tail -1 "$OUT/pytest_engine.log"
for i in 1 2 3; do
  run bs128_none$i FDT_LAZY_STATS=0 python bench.py --steps 40 --warmup 5 --global-batch 128
  run bs128_elem$i FDT_LAZY_SCOPE=elementwise python bench.py --steps 40 --warmup 5 --global-batch 128
  run bs128_all$i FDT_LAZY_SCOPE=all python bench.py --steps 40 --warmup 5 --global-batch 128
done
run bs1024_none FDT_LAZY_STATS=0 python bench.py --steps 30 --warmup 8
run bs1024_elem FDT_LAZY_SCOPE=elementwise python bench.py --steps 30 --warmup 8
echo done
