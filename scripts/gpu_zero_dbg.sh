#!/usr/bin/env bash
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/${1:-zero_dbg}
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu "tests/test_distributed_gpu.py::test_sharded_ngd_allreduce_between_graph_segments" tests/test_conv_kernels.py tests/test_resnet_engine.py tests/test_deterministic.py > "$OUT/a.log" 2>&1; echo "rc=$?"
tail -2 "$OUT/a.log"
exit 0
