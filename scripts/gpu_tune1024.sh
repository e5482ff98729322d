#!/usr/bin/env bash
# Re-tune the batch-1024 conv tile table, A/B the bench, engine tests with the new table.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${1:-tune1024}
mkdir -p "$OUT"
timeout -k 10 840 python -u scripts/tune_conv.py --batches 1024 --out "$OUT/tuned.json" > "$OUT/tune.log" 2>&1 || { echo tune failed; tail -5 "$OUT/tune.log"; exit 1; }
tail -1 "$OUT/tune.log"
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > "$OUT/bench1024_old.log" 2>&1 || exit 1
cp "$OUT/tuned.json" faster_distributed_training_amd/ops/conv_tuned.json
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > "$OUT/bench1024_new.log" 2>&1 || exit 1
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > "$OUT/bench1024_new2.log" 2>&1 || exit 1
grep -h '"value"' "$OUT"/bench*.log | python3 -c "import sys,json; [print(json.loads(l)['config']['global_batch'], json.loads(l)['ms_per_step']) for l in sys.stdin]"
timeout -k 10 400 python -u -m pytest tests/test_conv_kernels.py tests/test_resnet_engine.py tests/test_deterministic.py -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1; tail -2 "$OUT/pytest.log"
