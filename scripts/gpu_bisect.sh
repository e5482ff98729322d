#!/usr/bin/env bash
# Run one GPU test in each bisect worktree (.bisect/<commit>).
set -o pipefail
cd "$(dirname "$0")/.."
OUT=$PWD/gpurun_out/${1:-bisect}
mkdir -p "$OUT"
T="tests/test_distributed_gpu.py::test_sharded_ngd_allreduce_between_graph_segments"
for d in .bisect/*/; do
  c=$(basename $d)
  (cd $d && timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu "$T" > "$OUT/$c.log" 2>&1); echo "$c rc=$?"
done
exit 0
