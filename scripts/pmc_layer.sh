#!/usr/bin/env bash
# PMC counter passes for one conv layer (scripts/prof_layer.py). Counters are collected in
# runs of their own with --kernel-trace only (no sys/runtime trace).
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/pmc_$1; shift
mkdir -p "$OUT"
i=0
for grp in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_VALU_MFMA_BUSY_CYCLES" \
           "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_WAVES SQ_INSTS_SALU" \
           "MfmaUtil OccupancyPercent" "FETCH_SIZE" "WRITE_SIZE TCC_HIT_sum"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d "$OUT/p$i" -o run --pmc $grp -- python scripts/prof_layer.py "$@" > "$OUT/p$i.log" 2>&1 || { echo "pass $i failed"; exit 1; }
done
echo ok
