#!/usr/bin/env bash
# Round 5: per-layer K-loop form (rotated 2-deep prefetch vs legacy) chosen under graph replay,
# then benches with the chosen table.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r5f}
mkdir -p "$OUT"
cp faster_distributed_training_amd/ops/conv_tuned.json "$OUT/conv_tuned_before.json"
run() {
  local name=$1; shift
  timeout -k 10 300 env "$@" > "$OUT/$name.log" 2>&1 || { echo "$name failed"; tail -5 "$OUT/$name.log"; exit 1; }
  grep -h '"value"' "$OUT/$name.log" > "$OUT/$name.json"
  echo "$name $(grep -o '"ms_per_step": [0-9.]*' "$OUT/$name.json")"
}
run bs1024_legacy python bench.py --steps 30 --warmup 8
run bs128_legacy python bench.py --steps 40 --warmup 5 --global-batch 128
timeout -k 10 900 python -u scripts/retune_graph.py --loops --keys scripts/engine_keys/keys1024.txt scripts/engine_keys/keys128.txt \
  --ops fwd,dgrad --reps 10 --out "$OUT/conv_tuned.json" > "$OUT/retune_loops.log" 2>&1 || { echo retune failed; tail -20 "$OUT/retune_loops.log"; exit 1; }
grep -c " -> rot" "$OUT/retune_loops.log"; grep -c " -> old" "$OUT/retune_loops.log"
cp "$OUT/conv_tuned.json" faster_distributed_training_amd/ops/conv_tuned.json
run() {
  local name=$1; shift
  timeout -k 10 300 env "$@" > "$OUT/$name.log" 2>&1 || { echo "$name failed"; tail -5 "$OUT/$name.log"; exit 1; }
  grep -h '"value"' "$OUT/$name.log" > "$OUT/$name.json"
  echo "$name $(grep -o '"ms_per_step": [0-9.]*' "$OUT/$name.json")"
}
run bs1024_tuned python bench.py --steps 30 --warmup 8
run bs128_tuned python bench.py --steps 40 --warmup 5 --global-batch 128
run bs1024_allrot FDT_CONV_LOOP=rot python bench.py --steps 30 --warmup 8
run bs128_allrot FDT_CONV_LOOP=rot python bench.py --steps 40 --warmup 5 --global-batch 128
run bs1024_tuned2 python bench.py --steps 30 --warmup 8
run bs128_tuned2 python bench.py --steps 40 --warmup 5 --global-batch 128
echo done
