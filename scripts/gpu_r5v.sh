#!/usr/bin/env bash
# Transformer: NGD optimizer step replayed as HIP graphs at world 1 (B=32 / B=256) vs eager.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r5v}
mkdir -p "$OUT"
FDT_NATIVE=1 timeout -k 10 120 python -c "from faster_distributed_training_amd.ops import _native; _native.native()" || { echo "native extension stale or missing"; exit 1; }
run() {
  local name=$1; shift
  timeout -k 10 300 python bench.py "$@" > "$OUT/$name.log" 2>&1 || { echo "$name failed"; tail -5 "$OUT/$name.log"; exit 1; }
  grep -h '"value"' "$OUT/$name.log" > "$OUT/$name.json"
  echo "$name $(grep -o '"ms_per_step": [0-9.]*' "$OUT/$name.json") $(grep -o '"host_ms_per_step": [0-9.]*' "$OUT/$name.json") $(grep -o '"ngd_graph_replays": [0-9]*' "$OUT/$name.json")"
}
for rep in a b; do
FDT_NGD_GRAPHS=0 run tr_b32_eager_$rep --model transformer --global-batch 32 --steps 40 --warmup 12
FDT_NGD_GRAPHS=1 run tr_b32_graphs_$rep --model transformer --global-batch 32 --steps 40 --warmup 12
done
FDT_NGD_GRAPHS=0 run tr_b256_eager --model transformer --steps 20 --warmup 12
FDT_NGD_GRAPHS=1 run tr_b256_graphs --model transformer --steps 20 --warmup 12
echo done
