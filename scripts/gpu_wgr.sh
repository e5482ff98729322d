#!/usr/bin/env bash
# wgrad split-K reduce rewrite: kernel + engine tests, bs128 / bs1024 bench, bs128 timeline.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${1:-wgr}
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests/test_conv_kernels.py tests/test_deterministic.py tests/test_resnet_engine.py tests/test_gpu_kernels.py tests/test_distributed_gpu.py -m gpu -v -p no:cacheprovider --timeout 200 --timeout-method thread > "$OUT/pytest.log" 2>&1; rc=$?
tail -2 "$OUT/pytest.log"
case $rc in 0|1) ;; *) echo "pytest aborted rc=$rc"; exit 1;; esac
grep -E "^(FAILED|ERROR)" "$OUT/pytest.log" | head -20
run() {
  local name=$1; shift
  timeout -k 10 300 python bench.py "$@" > "$OUT/$name.log" 2>&1 || { echo "$name failed"; tail -5 "$OUT/$name.log"; exit 1; }
  grep -h '"value"' "$OUT/$name.log" > "$OUT/$name.json"
  echo "$name $(grep -o '"ms_per_step": [0-9.]*' "$OUT/$name.json")"
}
run b128 --steps 40 --warmup 5 --global-batch 128
run b1024 --steps 20 --warmup 5
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/prof128" -o run -- python3 bench.py --steps 4 --warmup 3 --global-batch 128 > "$OUT/prof128.log" 2>&1 || { echo prof failed; tail "$OUT/prof128.log"; exit 1; }
f=$(find "$OUT/prof128" -name '*kernel_trace.csv' | head -n 1)
python scripts/ktrace_step.py "$f" > "$OUT/timeline128.txt"
head -1 "$OUT/timeline128.txt"
grep wgrad_reduce "$OUT/timeline128.txt" | head -20
