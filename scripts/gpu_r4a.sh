#!/usr/bin/env bash
# Round 4 first call: HIP-graph/RCCL semantics probe, HEAD baselines (bs1024, bs128, bs128 --ddp),
# and a kernel-trace timeline of the DDP path at batch 128 (RCCL on its own queue).
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r4a}
mkdir -p "$OUT"
timeout -k 10 180 python -u scripts/graph_comm_probe.py > "$OUT/probe.log" 2>&1; rc=$?
cat "$OUT/probe.log" | tail -12
[ $rc -eq 0 ] || { echo "probe rc=$rc"; exit 1; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_prefetch.py -m gpu -q -k "mixup or prefetch or staging or submit" -p no:cacheprovider --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1; rc=$?
tail -2 "$OUT/pytest.log"
case $rc in 0|1|5) ;; *) echo "pytest aborted rc=$rc"; exit 1;; esac
run() {
  local name=$1; shift
  timeout -k 10 300 python bench.py "$@" > "$OUT/$name.log" 2>&1 || { echo "$name failed"; tail -5 "$OUT/$name.log"; exit 1; }
  grep -h '"value"' "$OUT/$name.log" > "$OUT/$name.json"
  echo "$name $(grep -o '"ms_per_step": [0-9.]*' "$OUT/$name.json") $(grep -o '"host_ms_per_step": [0-9.]*' "$OUT/$name.json")"
}
run bs1024 --steps 30 --warmup 5
run bs128 --steps 40 --warmup 5 --global-batch 128
run bs128_ddp --steps 40 --warmup 5 --global-batch 128 --ddp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/prof" -o run -- python3 bench.py --steps 4 --warmup 3 --global-batch 128 --ddp > "$OUT/prof.log" 2>&1 || { echo prof failed; tail "$OUT/prof.log"; exit 1; }
f=$(find "$OUT/prof" -name '*kernel_trace.csv' | head -n 1)
python scripts/ktrace_step.py "$f" > "$OUT/timeline_ddp128.txt"
head -1 "$OUT/timeline_ddp128.txt"
echo done
