#!/usr/bin/env bash
# A/B of the residual-join backward kernel: engine numerics, then kernel-trace profiles at the
# per-GPU batches of the 1- and 8-GPU scaling points for several block-count targets.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${1:-ab_rab}
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest tests/test_resnet_engine.py -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { echo pytest failed; exit 1; }
for nb in 1024 512 2048; do
  for gb in 128 1024; do
    FDT_RAB_BLOCKS=$nb timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/p${nb}_$gb" -o run -- python bench.py --steps 4 --warmup 3 --global-batch $gb > "$OUT/p${nb}_$gb.log" 2>&1 || { echo prof failed; exit 1; }
  done
done
FDT_RAB_BLOCKS=1024 timeout -k 10 300 python bench.py --steps 30 --warmup 5 --global-batch 128 > "$OUT/bench128.log" 2>&1 || { echo bench failed; exit 1; }
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > "$OUT/bench.log" 2>&1 || { echo bench failed; exit 1; }
echo done
