#!/usr/bin/env bash
# Round 4: re-tune exactly the conv-table entries one engine step consults (graph-replay
# timing), then bench with the new table.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r4n}
mkdir -p "$OUT"
for b in 1024 128; do
  timeout -k 10 200 python -u scripts/engine_launch_keys.py --batch $b > "$OUT/keys$b.txt" 2>&1 || { echo keys failed; tail -5 "$OUT/keys$b.txt"; exit 1; }
done
timeout -k 10 900 python -u scripts/retune_graph.py --keys "$OUT/keys1024.txt" "$OUT/keys128.txt" --ops wgrad,fwd,dgrad \
  --out faster_distributed_training_amd/ops/conv_tuned.json > "$OUT/retune.log" 2>&1 || { echo retune failed; tail -5 "$OUT/retune.log"; exit 1; }
grep -E "REPLACED|batch " "$OUT/retune.log" | tail -60
cp faster_distributed_training_amd/ops/conv_tuned.json "$OUT/conv_tuned.json"
run() {
  local name=$1; shift
  timeout -k 10 300 python bench.py "$@" > "$OUT/$name.log" 2>&1 || { echo "$name failed"; tail -5 "$OUT/$name.log"; exit 1; }
  grep -h '"value"' "$OUT/$name.log" > "$OUT/$name.json"
  echo "$name $(grep -o '"ms_per_step": [0-9.]*' "$OUT/$name.json")"
}
run bs1024 --steps 30 --warmup 8
run bs128 --steps 40 --warmup 5 --global-batch 128
run bs128_ddp --steps 40 --warmup 5 --global-batch 128 --ddp
echo done
