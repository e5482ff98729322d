#!/usr/bin/env bash
# Round 4: every README bench row at HEAD, one box.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r4final}
mkdir -p "$OUT"
run() {
  local name=$1; shift
  timeout -k 10 300 python bench.py "$@" > "$OUT/$name.log" 2>&1 || { echo "$name failed"; tail -5 "$OUT/$name.log"; exit 1; }
  grep -h '"value"' "$OUT/$name.log" > "$OUT/$name.json"
  echo "$name $(grep -o '"ms_per_step": [0-9.]*' "$OUT/$name.json") $(grep -o '"host_ms_per_step": [0-9.]*' "$OUT/$name.json")"
}
run bs1024 --steps 30 --warmup 8
run bs128 --steps 40 --warmup 5 --global-batch 128
run bs128_ddp --steps 40 --warmup 5 --global-batch 128 --ddp
run ngd_meta --ngd --meta_learning --steps 20 --warmup 12
run ngd_meta_sharded --ngd --meta_learning --sharded-ngd --steps 20 --warmup 12
run fsdp_full --fsdp --steps 20 --warmup 8
run fsdp_sgo --fsdp --fsdp-schedule shard_grad_op --steps 20 --warmup 8
run tr_b256 --model transformer --steps 20 --warmup 12
run tr_b32 --model transformer --global-batch 32 --steps 40 --warmup 12
run tr_fsdp --model transformer --fsdp --steps 20 --warmup 12
run no_native_bs1024 --no-native --steps 5 --warmup 2
echo done
