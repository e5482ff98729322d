#!/usr/bin/env bash
# Fused classifier head: engine / graph / distributed GPU tests, bench A/B (FDT_FUSED_HEAD),
# and the bs128 step timeline.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${1:-head}
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests/test_resnet_engine.py tests/test_ngd_graphs.py tests/test_distributed_gpu.py -m gpu -v -p no:cacheprovider --timeout 200 --timeout-method thread > "$OUT/pytest.log" 2>&1; rc=$?
tail -3 "$OUT/pytest.log"
case $rc in 0|1) ;; *) echo "pytest aborted rc=$rc"; exit 1;; esac
grep -E "^(FAILED|ERROR)" "$OUT/pytest.log" | head -20
run() {  # name, env value, args...
  local name=$1 fh=$2; shift 2
  FDT_FUSED_HEAD=$fh timeout -k 10 300 python bench.py "$@" > "$OUT/$name.log" 2>&1 || { echo "$name failed"; tail -5 "$OUT/$name.log"; exit 1; }
  grep -h '"value"' "$OUT/$name.log" > "$OUT/$name.json"
  echo "$name $(grep -o '"ms_per_step": [0-9.]*' "$OUT/$name.json") $(grep -o '"host_ms_per_step": [0-9.]*' "$OUT/$name.json")"
}
run b128_on 1 --steps 40 --warmup 5 --global-batch 128
run b128_off 0 --steps 40 --warmup 5 --global-batch 128
run b128_on2 1 --steps 40 --warmup 5 --global-batch 128
run b1024_on 1 --steps 20 --warmup 5
run b1024_off 0 --steps 20 --warmup 5
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/prof128" -o run -- python3 bench.py --steps 4 --warmup 3 --global-batch 128 > "$OUT/prof128.log" 2>&1 || { echo prof failed; tail "$OUT/prof128.log"; exit 1; }
f=$(find "$OUT/prof128" -name '*kernel_trace.csv' | head -n 1)
python scripts/ktrace_step.py "$f" > "$OUT/timeline128.txt"
head -1 "$OUT/timeline128.txt"
