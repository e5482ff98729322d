#!/usr/bin/env bash
# Round 6: halo-loop repeatability (bitwise, deterministic mode), the FSDP offload NGD
# optimizer-input diagnostic, and the sharded-NGD world-2 test per halo staging.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r6k}
mkdir -p "$OUT"
FDT_NATIVE=1 timeout -k 10 120 python -c "from faster_distributed_training_amd.ops import _native; _native.native()" || { echo "native extension stale or missing"; exit 1; }
timeout -k 10 300 python -u scripts/h3_repeat.py --reps 20 > "$OUT/h3_repeat.txt" 2>&1 || { echo "h3_repeat failed"; tail -20 "$OUT/h3_repeat.txt"; exit 1; }
grep -v amdgpu.ids "$OUT/h3_repeat.txt" | grep -v "mismatches 0/19, statistics mismatches 0/19"
timeout -k 10 400 python -u scripts/diag_offload_ngd.py > "$OUT/diag_offload_ngd.txt" 2>&1; echo "diag rc=$?"; grep -E "step|worst" "$OUT/diag_offload_ngd.txt"
for env in "FDT_CONV_H3_LOOP=reg" "FDT_CONV_H3_LOOP=dma1"; do
  env $env timeout -k 10 600 python -u -m pytest tests/test_distributed_gpu.py -m gpu -q -p no:cacheprovider --timeout 500 --timeout-method thread -k "test_sharded_ngd_graphs_world2" > "$OUT/pytest_zero_$env.log" 2>&1; echo "$env rc=$?"; grep -E "AssertionError: \(" "$OUT/pytest_zero_$env.log" | head -1
done
