#!/usr/bin/env bash
# Round 4: engine tests on the re-tuned table + per-layer rooflines of the calls the engine makes.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r4o}
mkdir -p "$OUT/pmc"
timeout -k 10 500 python -u -m pytest tests/test_resnet_engine.py tests/test_deterministic.py tests/test_distributed_gpu.py -m gpu -v -p no:cacheprovider \
  --timeout 200 --timeout-method thread > "$OUT/pytest.log" 2>&1; rc=$?
echo "pytest rc=$rc"; tail -1 "$OUT/pytest.log"
case $rc in 0) ;; 1) grep -E "^(FAILED|ERROR)" "$OUT/pytest.log" | head -20; exit 1;; *) echo aborted; exit 1;; esac
for b in 1024 128; do
  timeout -k 10 300 python scripts/roofline_layers.py --batch $b --keys profiles/r4/retune/keys$b.txt --md "$OUT/pmc/r4_bs${b}_roofline.md" --json "$OUT/pmc/roof$b.json" > "$OUT/roof$b.log" 2>&1 && tail -1 "$OUT/roof$b.log" || { tail -5 "$OUT/roof$b.log"; exit 1; }
done
echo done
