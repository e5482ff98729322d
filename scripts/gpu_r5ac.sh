#!/usr/bin/env bash
# World-8 sharded NGD balance sweep (per-axis cost, element slack), graphs on.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r5ac}
mkdir -p "$OUT"
for m in resnet50 transformer; do
for cfg in "200000:1.15" "400000:1.15" "200000:1.4" "400000:1.4" "800000:1.6"; do
  ac=${cfg%%:*}; sl=${cfg#*:}
  FDT_NGD_AXIS_COST=$ac FDT_NGD_SLACK=$sl timeout -k 10 300 python scripts/bench_ngd.py --model $m --world 8 --graphs > "$OUT/w8_${m}_${ac}_${sl}.txt" 2>&1 || { echo "failed $m $cfg"; tail -3 "$OUT/w8_${m}_${ac}_${sl}.txt"; exit 1; }
  echo "$m cost $ac slack $sl: $(tail -1 $OUT/w8_${m}_${ac}_${sl}.txt | sed 's/.*slowest rank: //')"
done
done
echo done
