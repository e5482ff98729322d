#!/usr/bin/env bash
# A/B at bs128: in-launch finalize on/off x old/new tile table; plus new DDP-graph tests.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r2h}
mkdir -p "$OUT"
B="--steps 40 --warmup 5 --global-batch 128"
for cfg in "--fuse-max 0 --table scripts/conv_tuned_r2a.json" "--fuse-max 512 --table scripts/conv_tuned_r2a.json" "--fuse-max 0" "--fuse-max 512" "--fuse-max 256"; do
  tag=$(echo "$cfg" | tr -c 'a-z0-9' '_')
  timeout -k 10 200 python scripts/ab_engine_cfg.py $cfg -- $B > "$OUT/ab_$tag.log" 2>&1 || { echo "ab $cfg failed"; exit 1; }
  echo "$cfg $(tail -1 $OUT/ab_$tag.log | python -c 'import json,sys; print(json.loads(sys.stdin.read())["ms_per_step"])')" >> "$OUT/ab.txt"
done
timeout -k 10 400 python -u -m pytest tests/test_distributed_gpu.py -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1; rc=$?; echo "pytest rc=$rc" >> "$OUT/pytest.log"
echo done
