#!/usr/bin/env bash
# Round 5: new / changed GPU tests, then HEAD benches + kernel traces.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r5b}
mkdir -p "$OUT"
timeout -k 10 900 python -u -m pytest -x -v -p no:cacheprovider --timeout 300 --timeout-method thread \
  tests/test_distributed_gpu.py -k "graph_comm or sharded_ngd_graphs or rccl_world1" > "$OUT/pytest_dist.log" 2>&1; rc=$?
echo "pytest dist rc=$rc"; tail -3 "$OUT/pytest_dist.log"
case $rc in 0|1) ;; *) echo aborted; exit 1;; esac
timeout -k 10 900 python -u -m pytest -x -v -s -p no:cacheprovider --timeout 400 --timeout-method thread \
  tests/test_convergence.py > "$OUT/pytest_conv.log" 2>&1; rc2=$?
echo "pytest conv rc=$rc2"; grep -E "^\{|passed|failed|Error" "$OUT/pytest_conv.log" | cut -c1-400 | tail -8
case $rc2 in 0|1) ;; *) echo aborted; exit 1;; esac
bash scripts/gpu_r5a.sh "${1:-r5b}_bench"
