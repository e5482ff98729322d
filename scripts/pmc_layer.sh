#!/usr/bin/env bash
# PMC passes on one conv layer through scripts/prof_layer.py (counters in runs of their own,
# --kernel-trace only).   bash scripts/pmc_layer.sh OUTDIR OP SHAPE [extra prof_layer args]
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/$1; OP=$2; SHAPE=$3; shift 3
mkdir -p "$OUT"
i=0
for grp in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_VALU_MFMA_BUSY_CYCLES" \
           "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_WAVES SQ_WAIT_INST_LDS" \
           "GRBM_GUI_ACTIVE GRBM_COUNT TCC_HIT_sum TCC_MISS_sum" "TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d "$OUT/L_p$i" -o run --pmc $grp -- python scripts/prof_layer.py --op $OP --shape $SHAPE --batch 1024 "$@" > "$OUT/L_p$i.log" 2>&1 || { echo "pass $i failed"; tail -5 "$OUT/L_p$i.log"; exit 1; }
done
python scripts/pmc_summary.py "$OUT" --match "fdt::" --arms L > "$OUT/summary.md"
grep -E "^## |MFMA busy|bank conflict share|SQ_WAIT_INST_LDS / |SQ_WAIT_ANY / |SQ_ACTIVE_INST_VMEM / |L2 hit|TCC_EA0" "$OUT/summary.md" | head -40
