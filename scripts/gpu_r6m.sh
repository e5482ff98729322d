#!/usr/bin/env bash
# Round 6: halo-loop repeatability with NaN-poisoned LDS and moving operand addresses.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r6m}
mkdir -p "$OUT"
FDT_NATIVE=1 timeout -k 10 120 python -c "from faster_distributed_training_amd.ops import _native; _native.native()" || { echo "native extension stale or missing"; exit 1; }
timeout -k 10 300 python -u scripts/h3_repeat.py --reps 12 > "$OUT/h3_repeat_poison.txt" 2>&1 || { echo "h3_repeat failed"; tail -20 "$OUT/h3_repeat_poison.txt"; exit 1; }
grep -v amdgpu.ids "$OUT/h3_repeat_poison.txt" | grep -v "mismatches 0/11, statistics mismatches 0/11, non-finite 0"
