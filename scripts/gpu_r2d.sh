#!/usr/bin/env bash
# Round-2 re-validation: GPU tests (incl. deterministic mode), smoke, benches (default and
# --deterministic cost), kernel-time profile of the bs1024 step.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r2d}
mkdir -p "$OUT"
timeout -k 10 700 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1; rc=$?; echo "pytest rc=$rc" >> "$OUT/pytest.log"
case $rc in 0|1) ;; *) echo "pytest aborted rc=$rc"; exit 1;; esac
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { echo smoke failed; exit 1; }
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > "$OUT/bench.log" 2>&1 || { echo bench failed; exit 1; }
timeout -k 10 300 python bench.py --steps 30 --warmup 5 --global-batch 128 > "$OUT/bench128.log" 2>&1 || { echo bench128 failed; exit 1; }
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --deterministic > "$OUT/bench_det.log" 2>&1 || { echo bench_det failed; exit 1; }
timeout -k 10 300 python bench.py --steps 30 --warmup 5 --global-batch 128 --deterministic > "$OUT/bench128_det.log" 2>&1 || { echo bench128_det failed; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof128" -o run -- python3 bench.py --steps 10 --warmup 3 --global-batch 128 > "$OUT/prof128.log" 2>&1 || { echo prof failed; exit 1; }
echo done
