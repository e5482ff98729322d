#!/usr/bin/env bash
# Hardware-counter roofline of one ResNet-50 training step (bench.py, eager launches so every
# dispatch is profiled individually).  One rocprofv3 pass per counter group (--kernel-trace
# only, never combined with sys/runtime tracing), plus one timing pass without counters.
#   bash scripts/pmc_step.sh <tag> <global-batch> [extra bench.py args]
# Then: python scripts/pmc_table.py gpurun_out/pmc_<tag>_<gb> --steps 4
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
TAG=$1; GB=$2; shift 2
OUT=gpurun_out/pmc_${TAG}_${GB}
mkdir -p "$OUT"
BENCH="bench.py --steps 2 --warmup 2 --no-graphs --global-batch $GB $*"
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d "$OUT/time" -o run -- python3 $BENCH > "$OUT/time.log" 2>&1 || { echo "timing pass failed"; exit 1; }
i=0
for grp in "FETCH_SIZE" \
           "WRITE_SIZE" \
           "SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_WAVES GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --kernel-trace --output-format csv -d "$OUT/p$i" -o run --pmc $grp -- python3 $BENCH > "$OUT/p$i.log" 2>&1 || { echo "pmc pass $i failed"; exit 1; }
done
echo ok
