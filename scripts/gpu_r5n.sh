#!/usr/bin/env bash
# Slot-row sweep (atomic contention of the statistics epilogues) at batch 1024 and 128.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r5n}
mkdir -p "$OUT"
FDT_NATIVE=1 timeout -k 10 120 python -c "from faster_distributed_training_amd.ops import _native; _native.native()" || { echo "native extension stale or missing"; exit 1; }
timeout -k 10 300 python -u scripts/conv_probe3.py --batch 1024 --rows 64,256,1024,4096,16384 > "$OUT/probe3_bs1024.txt" 2>&1 || { echo probe failed; tail -5 "$OUT/probe3_bs1024.txt"; exit 1; }
cat "$OUT/probe3_bs1024.txt"
timeout -k 10 300 python -u scripts/conv_probe3.py --batch 128 --rows 64,256,1024,2048 > "$OUT/probe3_bs128.txt" 2>&1 || { echo probe failed; tail -5 "$OUT/probe3_bs128.txt"; exit 1; }
cat "$OUT/probe3_bs128.txt"
echo done
