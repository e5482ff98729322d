#!/usr/bin/env bash
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${1:-last}
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1; rc=$?; echo "pytest rc=$rc" >> "$OUT/pytest.log"; tail -3 "$OUT/pytest.log"
case $rc in 0|1) ;; *) echo "pytest aborted rc=$rc"; exit 1;; esac
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { echo smoke failed; exit 1; }
tail -1 "$OUT/smoke.log"
timeout -k 10 300 python bench.py > "$OUT/bench_default.log" 2>&1 || { echo bench failed; exit 1; }
grep -h '"value"' "$OUT/bench_default.log" | cut -c1-160
