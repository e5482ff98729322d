#!/usr/bin/env bash
# Full GPU evidence: every -m gpu test, smoke, default bench.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${1:-full3}
mkdir -p "$OUT"
timeout -k 10 900 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1; rc=$?
echo "pytest rc=$rc" >> "$OUT/pytest.log"; tail -3 "$OUT/pytest.log"
case $rc in 0|1) ;; *) echo "pytest aborted rc=$rc"; exit 1;; esac
grep -E "^(FAILED|ERROR)" "$OUT/pytest.log" | head -20
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { echo smoke failed; tail "$OUT/smoke.log"; exit 1; }
tail -1 "$OUT/smoke.log"
timeout -k 10 300 python bench.py > "$OUT/bench.log" 2>&1 || { echo bench failed; tail "$OUT/bench.log"; exit 1; }
grep -h '"value"' "$OUT/bench.log" | cut -c1-200
echo done
