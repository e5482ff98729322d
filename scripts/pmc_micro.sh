#!/usr/bin/env bash
# Counter passes over one microbenchmark command (each pass its own rocprofv3 run, --kernel-trace only).
#   bash scripts/pmc_micro.sh <tag> <python args...>
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/pmcm_$1; shift
mkdir -p "$OUT"
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d "$OUT/time" -o run -- python3 "$@" > "$OUT/time.log" 2>&1 || { echo "time pass failed"; exit 1; }
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" \
           "SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_WAVES GRBM_GUI_ACTIVE" \
           "SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INST_CYCLES_VMEM_WR SQ_INST_CYCLES_VMEM_RD"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv -d "$OUT/p$i" -o run --pmc $grp -- python3 "$@" > "$OUT/p$i.log" 2>&1 || { echo "pmc pass $i failed"; exit 1; }
done
echo ok
