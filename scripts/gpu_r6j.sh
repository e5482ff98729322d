#!/usr/bin/env bash
# Round 6: 16-wave halo variant, the fixed h3 tests, the NGD offload diagnostic, and the
# sharded-NGD world-2 test under the CELU / halo switches.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r6j}
mkdir -p "$OUT"
FDT_NATIVE=1 timeout -k 10 120 python -c "from faster_distributed_training_amd.ops import _native; _native.native()" || { echo "native extension stale or missing"; exit 1; }
timeout -k 10 300 python -u scripts/bench_h3.py --batch 1024 > "$OUT/bench_h3_1024.txt" 2>&1 || { echo "bench_h3 failed"; tail -20 "$OUT/bench_h3_1024.txt"; exit 1; }
grep -v amdgpu.ids "$OUT/bench_h3_1024.txt"
timeout -k 10 600 python -u -m pytest tests/test_conv_kernels.py -m gpu -q -p no:cacheprovider --timeout 200 --timeout-method thread -k h3 > "$OUT/pytest_h3.log" 2>&1; rc=$?
echo "pytest h3 rc=$rc"; tail -1 "$OUT/pytest_h3.log"
case $rc in 0|1) ;; *) echo aborted; tail -20 "$OUT/pytest_h3.log"; exit 1;; esac
timeout -k 10 300 python -u scripts/diag_offload_ngd.py > "$OUT/diag_offload_ngd.txt" 2>&1; echo "diag rc=$?"; grep -v "amdgpu.ids\|Warning\|warn" "$OUT/diag_offload_ngd.txt" | tail -12
for env in "FDT_CELU_ZGRAD=1" "FDT_CELU_ZGRAD=0" "FDT_CONV_H3=0"; do
  env $env timeout -k 10 600 python -u -m pytest tests/test_distributed_gpu.py -m gpu -q -p no:cacheprovider --timeout 500 --timeout-method thread -k "test_sharded_ngd_graphs_world2" > "$OUT/pytest_zero_$env.log" 2>&1; echo "$env rc=$?"; grep -E "AssertionError: \(" "$OUT/pytest_zero_$env.log" | head -2
done
