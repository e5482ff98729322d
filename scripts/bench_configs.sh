#!/usr/bin/env bash
# The BASELINE.json configurations on one GPU (+ the eager "w/o tricks" ablations), one JSON
# line each under gpurun_out/configs/, and a bs-128 kernel profile.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/configs
mkdir -p "$OUT"
run() {  # name, args...
  local name=$1; shift
  timeout -k 10 300 python bench.py "$@" > "$OUT/$name.log" 2>&1 || { echo "$name failed"; tail -5 "$OUT/$name.log"; exit 1; }
  grep -h '"value"' "$OUT/$name.log" > "$OUT/$name.json"
  echo "$name $(grep -o '"ms_per_step": [0-9.]*' "$OUT/$name.json")"
}
run resnet50_bs1024 --steps 20 --warmup 5
run resnet50_bs512 --steps 20 --warmup 5 --global-batch 512
run resnet50_bs256 --steps 30 --warmup 5 --global-batch 256
run resnet50_bs128 --steps 30 --warmup 5 --global-batch 128
run ngd_meta --ngd --meta_learning --steps 20 --warmup 12
run fsdp --fsdp --steps 10 --warmup 3
run transformer --model transformer --steps 20 --warmup 12
run nonative --no-native --steps 5 --warmup 2
run tr_nonative --model transformer --no-native --steps 10 --warmup 12
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof128" -o run -- \
  python bench.py --steps 4 --warmup 3 --global-batch 128 > "$OUT/prof128.log" 2>&1 || { echo prof failed; exit 1; }
echo done
