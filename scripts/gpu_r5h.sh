#!/usr/bin/env bash
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r5h}
mkdir -p "$OUT"
timeout -k 10 400 python -u scripts/${2:-conv_probe}.py > "$OUT/conv_probe.txt" 2>&1 || { echo probe failed; tail -20 "$OUT/conv_probe.txt"; exit 1; }
cat "$OUT/conv_probe.txt"
