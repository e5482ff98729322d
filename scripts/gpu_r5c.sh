#!/usr/bin/env bash
# Round 5: lazy statistics (consumer-side BN finalize) -- engine numerics tests, then A/B benches.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r5c}
mkdir -p "$OUT"
timeout -k 10 900 python -u -m pytest -x -v -p no:cacheprovider --timeout 300 --timeout-method thread \
  tests/test_resnet_engine.py tests/test_deterministic.py > "$OUT/pytest_engine.log" 2>&1; rc=$?
echo "pytest engine rc=$rc"; tail -3 "$OUT/pytest_engine.log"
case $rc in 0) ;; 1) grep -E "^(FAILED|ERROR)|Error" "$OUT/pytest_engine.log" | head -20; exit 1;; *) echo aborted; exit 1;; esac
run() {
  local name=$1; shift
  timeout -k 10 300 env "$@" > "$OUT/$name.log" 2>&1 || { echo "$name failed"; tail -5 "$OUT/$name.log"; exit 1; }
  grep -h '"value"' "$OUT/$name.log" > "$OUT/$name.json"
  echo "$name $(grep -o '"ms_per_step": [0-9.]*' "$OUT/$name.json") $(grep -o '"host_ms_per_step": [0-9.]*' "$OUT/$name.json")"
}
for i in 1 2; do
run bs128_lazy$i FDT_LAZY_STATS=1 python bench.py --steps 40 --warmup 5 --global-batch 128
run bs128_nolazy$i FDT_LAZY_STATS=0 python bench.py --steps 40 --warmup 5 --global-batch 128
done
run bs1024_lazy FDT_LAZY_STATS=1 python bench.py --steps 30 --warmup 8
run bs1024_nolazy FDT_LAZY_STATS=0 python bench.py --steps 30 --warmup 8
run bs128_ddp FDT_LAZY_STATS=1 python bench.py --steps 40 --warmup 5 --global-batch 128 --ddp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_bs128" -o run -- python3 bench.py --steps 10 --warmup 5 --global-batch 128 > "$OUT/prof_bs128.log" 2>&1 || { echo prof failed; exit 1; }
f=$(find "$OUT/prof_bs128" -name '*kernel_stats.csv' | head -n 1); python scripts/kstats.py "$f" --steps 15 --top 70 > "$OUT/kstats_bs128.txt"; head -4 "$OUT/kstats_bs128.txt"
echo done
