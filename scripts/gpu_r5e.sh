#!/usr/bin/env bash
# Round 5: rotated conv K loop (true 2-deep prefetch) -- kernel tests, engine tests, benches, trace.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r5e}
mkdir -p "$OUT"
timeout -k 10 900 python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread \
  tests/test_conv_kernels.py tests/test_resnet_engine.py tests/test_deterministic.py tests/test_fused_epilogues.py > "$OUT/pytest.log" 2>&1; rc=$?
echo "pytest rc=$rc"; tail -2 "$OUT/pytest.log"
case $rc in 0) ;; 1) grep -E "^(FAILED|ERROR)|Error" "$OUT/pytest.log" | head -20; exit 1;; *) echo aborted; exit 1;; esac
run() {
  local name=$1; shift
  timeout -k 10 300 env "$@" > "$OUT/$name.log" 2>&1 || { echo "$name failed"; tail -5 "$OUT/$name.log"; exit 1; }
  grep -h '"value"' "$OUT/$name.log" > "$OUT/$name.json"
  echo "$name $(grep -o '"ms_per_step": [0-9.]*' "$OUT/$name.json")"
}
run bs128a python bench.py --steps 40 --warmup 5 --global-batch 128
run bs1024a python bench.py --steps 30 --warmup 8
run bs128b python bench.py --steps 40 --warmup 5 --global-batch 128
run bs1024b python bench.py --steps 30 --warmup 8
run bs128_ddp python bench.py --steps 40 --warmup 5 --global-batch 128 --ddp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_bs128" -o run -- python3 bench.py --steps 10 --warmup 5 --global-batch 128 > "$OUT/prof_bs128.log" 2>&1 || { echo prof failed; exit 1; }
f=$(find "$OUT/prof_bs128" -name '*kernel_stats.csv' | head -n 1); python scripts/kstats.py "$f" --steps 15 --top 70 > "$OUT/kstats_bs128.txt"; head -2 "$OUT/kstats_bs128.txt"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_bs1024" -o run -- python3 bench.py --steps 4 --warmup 3 > "$OUT/prof_bs1024.log" 2>&1 || { echo prof failed; exit 1; }
f=$(find "$OUT/prof_bs1024" -name '*kernel_stats.csv' | head -n 1); python scripts/kstats.py "$f" --steps 7 --top 70 > "$OUT/kstats_bs1024.txt"; head -2 "$OUT/kstats_bs1024.txt"
echo done
