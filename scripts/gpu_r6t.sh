#!/usr/bin/env bash
# Round 6: per-layer roofline tables at the final tree + the capture-check tests with the
# watchdog drain.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r6t}
mkdir -p "$OUT"
FDT_NATIVE=1 timeout -k 10 120 python -c "from faster_distributed_training_amd.ops import _native; _native.native()" || { echo "native extension stale or missing"; exit 1; }
timeout -k 10 600 python -u -m pytest tests/test_distributed_gpu.py -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread -k "graph_comm or allreduce_between or ddp" > "$OUT/pytest_comm.log" 2>&1; rc=$?
echo "pytest comm rc=$rc"; tail -1 "$OUT/pytest_comm.log"
case $rc in 0|1) grep -E "^(FAILED|ERROR)" "$OUT/pytest_comm.log" | head;; *) echo aborted; tail -20 "$OUT/pytest_comm.log"; exit 1;; esac
for b in 1024 128; do
  timeout -k 10 500 python -u scripts/roofline_layers.py --batch $b --md "$OUT/r6_bs${b}_roofline.md" > "$OUT/roofline_$b.log" 2>&1 || { echo "roofline $b failed"; tail -10 "$OUT/roofline_$b.log"; exit 1; }
  grep -i "total\|overall\|% of bound" "$OUT/r6_bs${b}_roofline.md" | tail -3
done
