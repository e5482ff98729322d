#!/usr/bin/env bash
# Rehearsal of the multi-rank bench paths on the one-GPU box (gloo ranks sharing cuda:0: correctness only,
# the times are not meaningful): dp (default), sharded NGD + meta, transformer, FSDP.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r5ad}
mkdir -p "$OUT"
export FDT_DIST_BACKEND=gloo
run() {
  local name=$1; shift
  timeout -k 10 400 python bench.py "$@" > "$OUT/$name.log" 2>&1 || { echo "$name failed"; tail -8 "$OUT/$name.log"; exit 1; }
  grep -h '"value"' "$OUT/$name.log" > "$OUT/$name.json"
  echo "$name $(grep -o '"n_gpus": [0-9]*' "$OUT/$name.json") $(grep -o '"dist_world": [0-9]*' "$OUT/$name.json") $(grep -o '"graph_comm": "[^"]*"' "$OUT/$name.json") $(grep -o '"ms_per_step": [0-9.]*' "$OUT/$name.json")"
}
run dp4 --gpus 4 --steps 4 --warmup 4
run ngd_meta4 --gpus 4 --ngd --meta_learning --sharded-ngd --steps 3 --warmup 12
run tr4 --gpus 4 --model transformer --steps 3 --warmup 4
run fsdp4 --gpus 4 --fsdp --steps 3 --warmup 3
echo done
