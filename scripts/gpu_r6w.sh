#!/usr/bin/env bash
# Round 6: transformer linear weight gradients at the 8-GPU share: split-K library bmm + slab
# sum vs the MFMA weight-gradient kernel (1x1 over tokens, direct fp32-atomic splits).
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r6w}
mkdir -p "$OUT"
timeout -k 10 300 python -u scripts/linear_wgrad_probe.py > "$OUT/linear_wgrad_probe.txt" 2>&1 || { echo "probe failed"; tail -10 "$OUT/linear_wgrad_probe.txt"; exit 1; }
grep -v amdgpu.ids "$OUT/linear_wgrad_probe.txt" | sed 's/  (/\n   (/g' | grep "^M\|best" | head -20
