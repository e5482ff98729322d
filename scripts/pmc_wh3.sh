#!/usr/bin/env bash
# PMC passes on the 16x16 128->128 3x3 weight gradient: halo loop vs the implicit GEMM.
# Counters in runs of their own with --kernel-trace only.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${1:-pmc_wh3}
mkdir -p "$OUT"
i=0
for arm in wh3 igemm; do
  if [ $arm = wh3 ]; then KG=9; else KG=0; fi
  for grp in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_VALU_MFMA_BUSY_CYCLES" \
             "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_WAVES SQ_WAIT_INST_LDS" \
             "GRBM_GUI_ACTIVE GRBM_COUNT TCC_HIT_sum TCC_MISS_sum"; do
    i=$((i+1))
    timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d "$OUT/${arm}_p$i" -o run --pmc $grp -- python scripts/prof_layer.py --op wgrad_plain --kg $KG --shape 16,128,128,3,1,1 --batch 1024 > "$OUT/${arm}_p$i.log" 2>&1 || { echo "pass $arm $i failed"; tail -5 "$OUT/${arm}_p$i.log"; exit 1; }
  done
done
python scripts/pmc_summary.py "$OUT" --match wh3_kernel --arms wh3 > "$OUT/summary_wh3.md" && python scripts/pmc_summary.py "$OUT" --match wgrad_kernel --arms igemm > "$OUT/summary_igemm.md"
grep -E "^## |MFMA busy|bank conflict share|SQ_WAIT_INST_LDS / |SQ_WAIT_ANY / |SQ_ACTIVE_INST_LDS / |L2 hit|SQ_INSTS_LDS:|SQ_INSTS_MFMA:" "$OUT/summary_wh3.md" "$OUT/summary_igemm.md"
echo pmc ok
