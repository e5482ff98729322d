#!/usr/bin/env bash
# Counter calibration (tools/pmc_calib.hip): known-bytes streams and a known-FLOP MFMA loop
# under one rocprofv3 pass per counter group -> gpurun_out/pmc_calib/{time,p1,p2,p3}.
#   hipcc -O3 --offload-arch=gfx950 tools/pmc_calib.hip -o tools/pmc_calib   (on the CPU host)
#   bash scripts/pmc_calib.sh && python scripts/pmc_calib_table.py gpurun_out/pmc_calib
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/pmc_calib
mkdir -p "$OUT"
timeout -k 10 120 ./tools/pmc_calib > "$OUT/run.log" 2>&1 || { cat "$OUT/run.log"; exit 1; }
cat "$OUT/run.log"
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d "$OUT/time" -o run -- ./tools/pmc_calib > "$OUT/time.log" 2>&1 || { echo "timing pass failed"; exit 1; }
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv -d "$OUT/p$i" -o run --pmc $grp -- ./tools/pmc_calib > "$OUT/p$i.log" 2>&1 || { echo "pmc pass $i failed"; exit 1; }
done
echo ok
