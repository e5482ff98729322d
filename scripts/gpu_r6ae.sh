#!/usr/bin/env bash
# Round 6: re-tune the batch-128 weight-gradient launches under graph replay (finer split grid),
# then A/B the step with the new table.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r6ae}
mkdir -p "$OUT"
cp faster_distributed_training_amd/ops/conv_tuned.json "$OUT/conv_tuned_before.json"
FDT_RETUNE_FINE=1 timeout -k 10 900 python -u scripts/retune_graph.py --batches ${BATCHES:-128} --ops ${OPS:-wgrad} --out "$OUT/conv_tuned.json" > "$OUT/retune.log" 2>&1 || { echo "retune failed"; tail -10 "$OUT/retune.log"; exit 1; }
grep -c REPLACED "$OUT/retune.log"; grep REPLACED "$OUT/retune.log" | head -20
j() { grep -h '"value"' "$OUT/$1.log" > "$OUT/$1.json"; echo "$1 $(grep -o '"ms_per_step": [0-9.]*' $OUT/$1.json)"; }
for v in new old new old; do
  if [ $v = new ]; then cp "$OUT/conv_tuned.json" faster_distributed_training_amd/ops/conv_tuned.json; else cp "$OUT/conv_tuned_before.json" faster_distributed_training_amd/ops/conv_tuned.json; fi
  timeout -k 10 300 python bench.py --global-batch ${GB:-128} --steps 40 > "$OUT/bs128_$v.log" 2>&1 || { echo "bench failed"; exit 1; }
  j bs128_$v
done
