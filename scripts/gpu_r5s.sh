#!/usr/bin/env bash
# Linear weight gradients: library split-K + slab sum vs the MFMA wgrad kernel (direct atomics).
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r5s}
mkdir -p "$OUT"
FDT_NATIVE=1 timeout -k 10 120 python -c "from faster_distributed_training_amd.ops import _native; _native.native()" || { echo "native extension stale or missing"; exit 1; }
timeout -k 10 300 python -u scripts/linear_wgrad_probe.py > "$OUT/linear_wgrad_probe.txt" 2>&1 || { echo probe failed; tail -5 "$OUT/linear_wgrad_probe.txt"; exit 1; }
cat "$OUT/linear_wgrad_probe.txt"
echo done
