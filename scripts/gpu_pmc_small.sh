#!/usr/bin/env bash
# Counters of latency-bound small-M convs at batch 128 (stage 3 / 4 shapes).
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${1:-pmcs}
mkdir -p "$OUT"
run() {  # name shape op
  local name=$1 shape=$2 op=$3
  mkdir -p "$OUT/$name"
  for grp in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_VALU_MFMA_BUSY_CYCLES" \
             "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAVES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU" \
             "TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum" ; do
    i=$((i+1))
    timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d "$OUT/$name/p$i" -o run --pmc $grp -- python scripts/prof_layer.py --op $op --shape $shape --batch 128 --reps 5 > "$OUT/$name/p$i.log" 2>&1 || { echo "$name pass $i failed"; tail "$OUT/$name/p$i.log"; exit 1; }
  done
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/$name/t" -o run -- python scripts/prof_layer.py --op $op --shape $shape --batch 128 --reps 20 > "$OUT/$name/t.log" 2>&1 || { echo "$name trace failed"; exit 1; }
}
i=0; run s3fwd 8,1024,256,1,1,0 fwd
i=0; run s4fwd 4,2048,512,1,1,0 fwd
i=0; run s3k3 8,256,256,3,1,1 fwd
i=0; run s3dg 8,256,1024,1,1,0 dgrad
echo done
