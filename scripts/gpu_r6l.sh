#!/usr/bin/env bash
# Round 6: NGD run-to-run sensitivity under FSDP offload; sharded-NGD world-2 divergence per step.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r6l}
mkdir -p "$OUT"
FDT_NATIVE=1 timeout -k 10 120 python -c "from faster_distributed_training_amd.ops import _native; _native.native()" || { echo "native extension stale or missing"; exit 1; }
timeout -k 10 500 python -u scripts/diag_offload_ngd.py > "$OUT/diag_offload_ngd.txt" 2>&1; echo "diag rc=$?"; grep -E "step|worst" "$OUT/diag_offload_ngd.txt"
timeout -k 10 600 python -u scripts/diag_sharded_h3.py > "$OUT/diag_sharded_h3.txt" 2>&1; echo "sharded h3 rc=$?"; grep -E "^step" "$OUT/diag_sharded_h3.txt"
FDT_CONV_H3=0 timeout -k 10 600 python -u scripts/diag_sharded_h3.py > "$OUT/diag_sharded_noh3.txt" 2>&1; echo "sharded noh3 rc=$?"; grep -E "^step" "$OUT/diag_sharded_noh3.txt"
