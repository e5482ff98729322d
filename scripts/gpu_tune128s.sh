#!/usr/bin/env bash
# Batch-128 tile re-tune with split-K up to 16, A/B bench, engine tests with the candidate table.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${1:-tune128s}
mkdir -p "$OUT"
timeout -k 10 840 python -u scripts/tune_conv.py --batches 128 --splits 1 2 4 8 16 --out "$OUT/tuned.json" > "$OUT/tune.log" 2>&1 || { echo tune failed; tail -5 "$OUT/tune.log"; exit 1; }
timeout -k 10 300 python bench.py --steps 30 --warmup 5 --global-batch 128 > "$OUT/old.log" 2>&1 || exit 1
cp "$OUT/tuned.json" faster_distributed_training_amd/ops/conv_tuned.json
timeout -k 10 300 python bench.py --steps 30 --warmup 5 --global-batch 128 > "$OUT/new.log" 2>&1 || exit 1
timeout -k 10 300 python bench.py --steps 30 --warmup 5 --global-batch 128 > "$OUT/new2.log" 2>&1 || exit 1
grep -h '"value"' "$OUT"/old.log "$OUT"/new.log "$OUT"/new2.log | python3 -c "import sys,json; [print(json.loads(l)['ms_per_step']) for l in sys.stdin]"
timeout -k 10 400 python -u -m pytest tests/test_conv_kernels.py tests/test_resnet_engine.py tests/test_deterministic.py -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1; tail -1 "$OUT/pytest.log"
