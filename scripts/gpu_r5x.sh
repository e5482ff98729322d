#!/usr/bin/env bash
# Round 5: 3x3 materialisation A/B, per-layer rooflines and the whole-step counter tables.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r5x}
mkdir -p "$OUT/pmc"
FDT_NATIVE=1 timeout -k 10 120 python -c "from faster_distributed_training_amd.ops import _native; _native.native()" || { echo "native extension stale or missing"; exit 1; }
run() {
  local name=$1; shift
  timeout -k 10 300 python bench.py "$@" > "$OUT/$name.log" 2>&1 || { echo "$name failed"; tail -5 "$OUT/$name.log"; exit 1; }
  grep -h '"value"' "$OUT/$name.log" > "$OUT/$name.json"
  echo "$name $(grep -o '"ms_per_step": [0-9.]*' "$OUT/$name.json")"
}
FDT_MATERIALIZE_3X3=1 run bs1024_m1 --steps 30 --warmup 8
FDT_MATERIALIZE_3X3=0 run bs1024_m0 --steps 30 --warmup 8
FDT_MATERIALIZE_3X3=1 run bs128_m1 --steps 40 --warmup 5 --global-batch 128
FDT_MATERIALIZE_3X3=0 run bs128_m0 --steps 40 --warmup 5 --global-batch 128
for b in 1024 128; do
  timeout -k 10 300 python scripts/roofline_layers.py --batch $b --md "$OUT/pmc/r5_bs${b}_roofline.md" --json "$OUT/pmc/r5_bs${b}_roofline.json" > "$OUT/roof$b.log" 2>&1 && tail -1 "$OUT/roof$b.log" || exit 1
done
for b in 1024 128; do
  bash scripts/pmc_step.sh r5 $b > "$OUT/pmc_step_$b.log" 2>&1 || { echo "pmc $b failed"; tail -3 "$OUT/pmc_step_$b.log"; exit 1; }
  python scripts/pmc_table.py gpurun_out/pmc_r5_$b --steps 4 --out "$OUT/pmc/r5_head_counters_bs$b.md" > /dev/null && head -6 "$OUT/pmc/r5_head_counters_bs$b.md"
done
echo done
