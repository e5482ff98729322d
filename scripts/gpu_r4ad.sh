#!/usr/bin/env bash
# Round 4: second, finer split-K pass of the graph-replay retune on the batch-1024 keys, then A/B.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r4ad}
mkdir -p "$OUT"
cp faster_distributed_training_amd/ops/conv_tuned.json "$OUT/conv_tuned_before.json"
run() {
  local name=$1; shift
  timeout -k 10 300 python bench.py "$@" > "$OUT/$name.log" 2>&1 || { echo "$name failed"; tail -5 "$OUT/$name.log"; exit 1; }
  grep -h '"value"' "$OUT/$name.log" > "$OUT/$name.json"
  echo "$name $(grep -o '"ms_per_step": [0-9.]*' "$OUT/$name.json")"
}
run b1024_before --steps 30 --warmup 8
FDT_RETUNE_FINE=1 timeout -k 10 1000 python -u scripts/retune_graph.py --keys scripts/engine_keys/keys1024.txt --ops wgrad,fwd,dgrad \
  --out faster_distributed_training_amd/ops/conv_tuned.json > "$OUT/retune.log" 2>&1 || { echo retune failed; tail -5 "$OUT/retune.log"; exit 1; }
grep -E "REPLACED|batch " "$OUT/retune.log" | tail -30
cp faster_distributed_training_amd/ops/conv_tuned.json "$OUT/conv_tuned.json"
run b1024_after --steps 30 --warmup 8
run b1024_after2 --steps 30 --warmup 8
echo done
