#!/usr/bin/env bash
# PMC passes on the 16x16 128->128 3x3 forward: halo loop (kg 5) vs the tuned implicit GEMM.
# Counters in runs of their own with --kernel-trace only.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${1:-pmc_h3}
mkdir -p "$OUT"
i=0
for arm in h3 tuned; do
  if [ $arm = h3 ]; then export FDT_CONV_H3=1; else export FDT_CONV_H3=0; fi
  for grp in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_VALU_MFMA_BUSY_CYCLES" \
             "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_WAVES SQ_WAIT_INST_LDS" \
             "GRBM_GUI_ACTIVE GRBM_COUNT TCC_HIT_sum TCC_MISS_sum" "TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum"; do
    i=$((i+1))
    timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d "$OUT/${arm}_p$i" -o run --pmc $grp -- python scripts/prof_layer.py --op fwd --pro none --shape 16,128,128,3,1,1 --batch 1024 > "$OUT/${arm}_p$i.log" 2>&1 || { echo "pass $arm $i failed"; tail -5 "$OUT/${arm}_p$i.log"; exit 1; }
  done
done
echo pmc ok
