#!/usr/bin/env bash
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${1:-halo}
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_conv_kernels.py -k "halo" > "$OUT/pytest_halo.log" 2>&1 || { echo pytest failed; tail -40 "$OUT/pytest_halo.log"; exit 1; }
tail -1 "$OUT/pytest_halo.log"
timeout -k 10 300 python scripts/bench_halo.py --batch 1024 > "$OUT/halo1024.txt" 2>&1 || { tail "$OUT/halo1024.txt"; exit 1; }
timeout -k 10 300 python scripts/bench_halo.py --batch 128 > "$OUT/halo128.txt" 2>&1 || { tail "$OUT/halo128.txt"; exit 1; }
cat "$OUT/halo1024.txt" "$OUT/halo128.txt"
