#!/usr/bin/env bash
# In-launch BN finalize for small conv grids + retuned batch-128 table: engine / conv /
# distributed GPU tests, benches at bs 128 and 1024, kernel trace of the bs128 step.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r2g}
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests/test_conv_kernels.py tests/test_resnet_engine.py tests/test_deterministic.py tests/test_distributed_gpu.py tests/test_fused_epilogues.py -m gpu -q -p no:cacheprovider --timeout 200 --timeout-method thread > "$OUT/pytest.log" 2>&1; rc=$?; echo "pytest rc=$rc" >> "$OUT/pytest.log"
case $rc in 0|1) ;; *) echo "pytest aborted rc=$rc"; exit 1;; esac
timeout -k 10 300 python bench.py --steps 30 --warmup 5 --global-batch 128 > "$OUT/bench128.log" 2>&1 || { echo bench128 failed; exit 1; }
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > "$OUT/bench.log" 2>&1 || { echo bench failed; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof128" -o run -- python3 bench.py --steps 10 --warmup 3 --global-batch 128 > "$OUT/prof128.log" 2>&1 || { echo prof failed; exit 1; }
echo done
