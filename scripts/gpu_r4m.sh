#!/usr/bin/env bash
# Round 4: conv table re-tuned under graph replay -- engine tests at the shipped configs,
# bs1024 / bs128 / DDP-bs128 benches, refreshed rooflines.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r4m}
mkdir -p "$OUT"
timeout -k 10 500 python -u -m pytest tests/test_resnet_engine.py tests/test_conv_kernels.py tests/test_deterministic.py -m gpu -v -p no:cacheprovider \
  --timeout 200 --timeout-method thread > "$OUT/pytest.log" 2>&1; rc=$?
echo "pytest rc=$rc"; tail -1 "$OUT/pytest.log"
case $rc in 0) ;; 1) grep -E "^(FAILED|ERROR)" "$OUT/pytest.log" | head -20; exit 1;; *) echo aborted; exit 1;; esac
run() {
  local name=$1; shift
  timeout -k 10 300 python bench.py "$@" > "$OUT/$name.log" 2>&1 || { echo "$name failed"; tail -5 "$OUT/$name.log"; exit 1; }
  grep -h '"value"' "$OUT/$name.log" > "$OUT/$name.json"
  echo "$name $(grep -o '"ms_per_step": [0-9.]*' "$OUT/$name.json")"
}
run bs1024 --steps 30 --warmup 8
run bs1024b --steps 30 --warmup 8
run bs128 --steps 40 --warmup 5 --global-batch 128
run bs128_ddp --steps 40 --warmup 5 --global-batch 128 --ddp
run ngd_meta --ngd --meta_learning --steps 20 --warmup 12
mkdir -p "$OUT/pmc"
for b in 1024 128; do
  timeout -k 10 300 python scripts/roofline_layers.py --batch $b --md "$OUT/pmc/r4_bs${b}_roofline.md" --json "$OUT/pmc/roof$b.json" > "$OUT/roof$b.log" 2>&1 && tail -1 "$OUT/roof$b.log" || exit 1
done
echo done
