#!/usr/bin/env bash
# Full GPU suite + smoke + benches (ResNet bs1024 / bs128, transformer) at this checkpoint.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r2l}
mkdir -p "$OUT"
timeout -k 10 800 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 200 --timeout-method thread > "$OUT/pytest.log" 2>&1; rc=$?; echo "pytest rc=$rc" >> "$OUT/pytest.log"
case $rc in 0|1) ;; *) echo "pytest aborted rc=$rc"; exit 1;; esac
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { echo smoke failed; exit 1; }
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > "$OUT/bench.log" 2>&1 || { echo bench failed; exit 1; }
timeout -k 10 300 python bench.py --steps 30 --warmup 5 --global-batch 128 > "$OUT/bench128.log" 2>&1 || { echo bench128 failed; exit 1; }
timeout -k 10 300 python bench.py --model transformer --steps 20 --warmup 12 > "$OUT/bench_tr.log" 2>&1 || { echo bench_tr failed; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_tr" -o run -- python3 bench.py --model transformer --steps 10 --warmup 12 --seq-buckets 256 > "$OUT/prof_tr.log" 2>&1 || { echo prof failed; exit 1; }
echo done
