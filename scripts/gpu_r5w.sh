#!/usr/bin/env bash
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r5w}
mkdir -p "$OUT"
timeout -k 10 300 python scripts/host_profile_tr.py --batch 32 > "$OUT/host_profile_tr_b32.txt" 2>&1 || { echo failed; tail -5 "$OUT/host_profile_tr_b32.txt"; exit 1; }
echo done
