#!/usr/bin/env bash
# Convergence test on held-out loss, twice (stability), plus the curves.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r5ab}
mkdir -p "$OUT"
for rep in 1 2; do
timeout -k 10 900 python -u -m pytest tests/test_convergence.py -m gpu -v -s -p no:cacheprovider --timeout 400 --timeout-method thread > "$OUT/pytest_$rep.log" 2>&1; rc=$?
echo "rep $rep rc=$rc $(tail -1 $OUT/pytest_$rep.log)"; grep -E "^(FAILED|ERROR)" "$OUT/pytest_$rep.log" | head; grep -oE "'engine_test_loss': [0-9.]+, 'reference_test_loss': [0-9.]+, 'bf16_torch_test_loss': [0-9.]+" "$OUT/pytest_$rep.log"
case $rc in 0|1) ;; *) exit 1;; esac
done
timeout -k 10 600 python scripts/convergence.py --opts madgrad,ngd --arch resnet18 --out "$OUT/convergence_resnet18.json" > "$OUT/convergence_resnet18.log" 2>&1 && tail -2 "$OUT/convergence_resnet18.log"
echo done
