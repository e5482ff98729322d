#!/usr/bin/env bash
# Round 6: sharded vs unsharded NGD per step, with the gradient norm, clipping on (10) and off.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r6o}
mkdir -p "$OUT"
FDT_NATIVE=1 timeout -k 10 120 python -c "from faster_distributed_training_amd.ops import _native; _native.native()" || { echo "native extension stale or missing"; exit 1; }
for c in 10 1e9; do
  CLIP=$c timeout -k 10 600 python -u scripts/diag_sharded_h3.py > "$OUT/diag_sharded_clip$c.txt" 2>&1; echo "clip $c rc=$?"; grep -E "^(step|arms)" "$OUT/diag_sharded_clip$c.txt"
done
