#!/usr/bin/env bash
# A/B of engine switches at bs128 and bs1024 (one bench per setting).
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/${1:-ab3}; shift
mkdir -p "$OUT"
for spec in "$@"; do
  name=${spec%%:*}; envs=${spec#*:}
  for gb in 128 1024; do
    st=30; [ $gb = 1024 ] && st=15
    env $envs timeout -k 10 300 python bench.py --steps $st --warmup 5 --global-batch $gb > "$OUT/${name}_$gb.log" 2>&1 || { echo "$name $gb failed"; tail -3 "$OUT/${name}_$gb.log"; exit 1; }
    echo "$name bs$gb $(grep -h '"value"' "$OUT/${name}_$gb.log" | python3 -c 'import sys,json; print(json.loads(sys.stdin.read())["ms_per_step"])')"
  done
done
