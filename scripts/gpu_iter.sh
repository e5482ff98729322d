#!/usr/bin/env bash
# Iteration GPU call: selected GPU tests, 1-GPU benches at bs 1024 / 128, kernel-time stats.
#   bash scripts/gpu_iter.sh <tag> [pytest selection...]
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
SEL=${*:-tests}
timeout -k 10 600 python -u -m pytest $SEL -m gpu -x -v -p no:cacheprovider --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1; rc=$?; echo "pytest rc=$rc" >> "$OUT/pytest.log"
[ $rc -eq 0 ] || { echo "pytest failed rc=$rc"; tail -30 "$OUT/pytest.log"; exit 1; }
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > "$OUT/bench.log" 2>&1 || { echo bench failed; tail -20 "$OUT/bench.log"; exit 1; }
timeout -k 10 300 python bench.py --steps 30 --warmup 5 --global-batch 128 > "$OUT/bench128.log" 2>&1 || { echo bench128 failed; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- python3 bench.py --steps 4 --warmup 3 > "$OUT/prof.log" 2>&1 || { echo prof failed; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof128" -o run -- python3 bench.py --steps 4 --warmup 3 --global-batch 128 > "$OUT/prof128.log" 2>&1 || { echo prof128 failed; exit 1; }
tail -1 "$OUT/bench.log"; tail -1 "$OUT/bench128.log"
echo done
