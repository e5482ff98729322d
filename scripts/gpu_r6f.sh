#!/usr/bin/env bash
# Round 6: halo-loop cost probe, then the remaining simulated world-8 ranks + transformer host profiles.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r6f}
mkdir -p "$OUT"
FDT_NATIVE=1 timeout -k 10 120 python -c "from faster_distributed_training_amd.ops import _native; _native.native()" || { echo "native extension stale or missing"; exit 1; }
timeout -k 10 300 python -u scripts/h3_probe.py --batch 1024 > "$OUT/h3_probe_1024.txt" 2>&1 || { echo "h3 probe failed"; tail -20 "$OUT/h3_probe_1024.txt"; exit 1; }
grep -v amdgpu.ids "$OUT/h3_probe_1024.txt"
NGD_RANKS="" bash scripts/gpu_r6c.sh "${1:-r6f}/sim"
