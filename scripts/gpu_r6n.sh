#!/usr/bin/env bash
# Round 6: which arm of the sharded-NGD world-2 comparison is not repeatable (halo loop on).
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r6n}
mkdir -p "$OUT"
FDT_NATIVE=1 timeout -k 10 120 python -c "from faster_distributed_training_amd.ops import _native; _native.native()" || { echo "native extension stale or missing"; exit 1; }
ARMS=0,0,1,1 timeout -k 10 900 python -u scripts/diag_sharded_h3.py > "$OUT/diag_sharded_repeat.txt" 2>&1; echo "rc=$?"; grep -E "^(step|arms)" "$OUT/diag_sharded_repeat.txt"
ARMS=1,1 FDT_NGD_OVERLAP=0 timeout -k 10 600 python -u scripts/diag_sharded_h3.py > "$OUT/diag_sharded_repeat_nooverlap.txt" 2>&1; echo "rc=$?"; grep -E "^(step|arms)" "$OUT/diag_sharded_repeat_nooverlap.txt"
