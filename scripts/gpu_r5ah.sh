#!/usr/bin/env bash
# Convergence test with repeated arms + the in-test fp32 spread.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r5ah}
mkdir -p "$OUT"
FDT_NATIVE=1 timeout -k 10 120 python -c "from faster_distributed_training_amd.ops import _native; _native.native()" || { echo "native extension stale or missing"; exit 1; }
timeout -k 10 900 python -u -m pytest tests/test_convergence.py -m gpu -v -s -p no:cacheprovider --timeout 400 --timeout-method thread > "$OUT/pytest.log" 2>&1; rc=$?
echo "pytest rc=$rc"; tail -1 "$OUT/pytest.log"; grep -E "^(FAILED|ERROR)|AssertionError|'reference_spread_loss'" "$OUT/pytest.log" | cut -c1-300 | head -20
grep -o "'engine_test_losses': [^]]*], [^]]*]" "$OUT/pytest.log" | head; grep -o "'reference_test_losses': [^]]*]" "$OUT/pytest.log"; grep -o "'bf16_torch_test_losses': [^]]*]" "$OUT/pytest.log"
echo done
