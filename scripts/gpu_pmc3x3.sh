#!/usr/bin/env bash
# Counters of the compute-bound 3x3 forward conv at batch 1024 (stage 1 and stage 3 shapes).
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${1:-pmc3}
mkdir -p "$OUT"
timeout -k 10 60 rocprofv3 --list-avail > "$OUT/avail.txt" 2>&1 || true
run() {  # name shape
  local name=$1 shape=$2; shift 2
  mkdir -p "$OUT/$name"
  local i=0
  for grp in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_VALU_MFMA_BUSY_CYCLES" \
             "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAVES SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS SQ_INSTS_SALU" \
             "TA_TA_BUSY_sum TA_BUFFER_READ_WAVEFRONTS_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum" \
             "TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE"; do
    i=$((i+1))
    timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d "$OUT/$name/p$i" -o run --pmc $grp -- python scripts/prof_layer.py --op fwd --shape $shape --batch 1024 --reps 5 --pro none "$@" > "$OUT/$name/p$i.log" 2>&1 || echo "$name pass $i failed (counter set?)"
  done
  timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d "$OUT/$name/t" -o run -- python scripts/prof_layer.py --op fwd --shape $shape --batch 1024 --reps 20 --pro none "$@" > "$OUT/$name/t.log" 2>&1 || { echo "$name trace failed"; exit 1; }
}
run s1k3 32,64,64,3,1,1
run s3k3 8,256,256,3,1,1
echo done
