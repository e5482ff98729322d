#!/usr/bin/env bash
# Reducer dedup of readiness signals + convergence tail median: distributed GPU tests + convergence tests.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r5aa}
mkdir -p "$OUT"
FDT_NATIVE=1 timeout -k 10 120 python -c "from faster_distributed_training_amd.ops import _native; _native.native()" || { echo "native extension stale or missing"; exit 1; }
timeout -k 10 1100 python -u -m pytest tests/test_distributed_gpu.py tests/test_convergence.py tests/test_transformer_graphs.py -m gpu -v -p no:cacheprovider --timeout 400 --timeout-method thread > "$OUT/pytest.log" 2>&1; rc=$?
echo "pytest rc=$rc"; tail -1 "$OUT/pytest.log"; grep -E "^(FAILED|ERROR)" "$OUT/pytest.log" | head; grep -E "^\{'optimizer'" "$OUT/pytest.log" | cut -c1-400
echo done
