#!/usr/bin/env bash
# Round 4: 3x3 convs normalising in their operand staging (FDT_MATERIALIZE_3X3=0) vs the
# materialised inputs, each on a table tuned for its own variant keys.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r4y}
mkdir -p "$OUT"
for b in 1024 128; do
  FDT_MATERIALIZE_3X3=0 timeout -k 10 200 python -u scripts/engine_launch_keys.py --batch $b > "$OUT/keys_nomat$b.txt" 2>&1 || { echo keys failed; tail -5 "$OUT/keys_nomat$b.txt"; exit 1; }
done
grep -E ":3:[12]:1 " "$OUT/keys_nomat1024.txt" | head -20
timeout -k 10 900 python -u scripts/retune_graph.py --keys "$OUT/keys_nomat1024.txt" "$OUT/keys_nomat128.txt" --ops wgrad,fwd,dgrad \
  --out faster_distributed_training_amd/ops/conv_tuned.json > "$OUT/retune.log" 2>&1 || { echo retune failed; tail -5 "$OUT/retune.log"; exit 1; }
grep -E "REPLACED|batch " "$OUT/retune.log" | tail -30
cp faster_distributed_training_amd/ops/conv_tuned.json "$OUT/conv_tuned.json"
run() {
  local name=$1; shift
  timeout -k 10 300 python bench.py "$@" > "$OUT/$name.log" 2>&1 || { echo "$name failed"; tail -5 "$OUT/$name.log"; exit 1; }
  grep -h '"value"' "$OUT/$name.log" > "$OUT/$name.json"
  echo "$name $(grep -o '"ms_per_step": [0-9.]*' "$OUT/$name.json")"
}
run b1024_mat --steps 30 --warmup 8
FDT_MATERIALIZE_3X3=0 run b1024_nomat --steps 30 --warmup 8
run b128_mat --steps 40 --warmup 5 --global-batch 128
FDT_MATERIALIZE_3X3=0 run b128_nomat --steps 40 --warmup 5 --global-batch 128
echo done
