#!/usr/bin/env bash
# Round 4: the whole GPU test suite at HEAD (one process), smoke, default bench.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r4l}
mkdir -p "$OUT"
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1; rc=$?
echo "pytest rc=$rc"; tail -1 "$OUT/pytest_gpu.log"
case $rc in 0) ;; 1) grep -E "^(FAILED|ERROR)" "$OUT/pytest_gpu.log" | head -20; exit 1;; *) echo aborted; tail -20 "$OUT/pytest_gpu.log"; exit 1;; esac
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 && echo smoke ok || { echo smoke failed; tail -5 "$OUT/smoke.log"; exit 1; }
timeout -k 10 300 python bench.py > "$OUT/bench_default.log" 2>&1 && grep '"value"' "$OUT/bench_default.log" | tail -1 || { tail -5 "$OUT/bench_default.log"; exit 1; }
echo done
