#!/usr/bin/env bash
# Round 6: hardware-counter tables of every kernel of one training step (batch 1024 / 128) at
# the final tree; tables built on the box, raw counter CSVs dropped.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
for gb in 1024 128; do
  bash scripts/pmc_step.sh r6 $gb > gpurun_out/pmc_r6_$gb.log 2>&1 || { echo "pmc $gb failed"; tail -5 gpurun_out/pmc_r6_$gb.log; exit 1; }
  python scripts/pmc_table.py gpurun_out/pmc_r6_$gb --steps 4 --top 45 --out gpurun_out/r6_head_counters_bs$gb.md > /dev/null || { echo "table $gb failed"; exit 1; }
  head -12 gpurun_out/r6_head_counters_bs$gb.md
  rm -rf gpurun_out/pmc_r6_$gb
done
