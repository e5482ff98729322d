#!/usr/bin/env bash
# One GPU round-trip: GPU tests, smoke, 1-GPU bench, kernel-level profile of the bench.
# Each GPU step has its own time limit; the chain stops at the first failure.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${1:-check}
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1; rc=$?; echo "pytest rc=$rc" >> "$OUT/pytest.log"
case $rc in 0|1) ;; *) echo "pytest aborted rc=$rc"; exit 1;; esac
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { echo smoke failed; exit 1; }
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > "$OUT/bench.log" 2>&1 || { echo bench failed; exit 1; }
timeout -k 10 300 python bench.py --steps 30 --warmup 5 --global-batch 128 > "$OUT/bench128.log" 2>&1 || { echo bench128 failed; exit 1; }
timeout -k 10 300 python bench.py --model transformer --steps 20 --warmup 12 > "$OUT/bench_tr.log" 2>&1 || { echo bench_tr failed; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- python bench.py --steps 4 --warmup 3 > "$OUT/prof.log" 2>&1 || { echo prof failed; exit 1; }
timeout -k 10 300 python resnet50_test.py --synthetic --bs 1024 --epoch 1 --steps 12 --no_eval --no_plot --profile_steps 8 --checkpoint_dir /tmp/ck > "$OUT/profile_steps.log" 2>&1 || { echo profile_steps failed; exit 1; }
echo done
