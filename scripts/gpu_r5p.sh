#!/usr/bin/env bash
# Residual join folded into the next 1x1 conv vs join pass + conv, per stage and tile.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r5p}
mkdir -p "$OUT"
FDT_NATIVE=1 timeout -k 10 120 python -c "from faster_distributed_training_amd.ops import _native; _native.native()" || { echo "native extension stale or missing"; exit 1; }
for b in 1024 128; do
timeout -k 10 300 python -u scripts/join_probe.py --batch $b > "$OUT/join_probe_bs$b.txt" 2>&1 || { echo probe failed; tail -5 "$OUT/join_probe_bs$b.txt"; exit 1; }
cat "$OUT/join_probe_bs$b.txt"
done
echo done
