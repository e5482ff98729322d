#!/usr/bin/env bash
# Round 6: CELU join derivative fix + halo 3x3 loop -- kernel tests against fp32 oracles,
# the halo-vs-tuned microbenchmark, then the ResNet-18 / MADGRAD convergence ablation.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r6a}
mkdir -p "$OUT"
FDT_NATIVE=1 timeout -k 10 120 python -c "from faster_distributed_training_amd.ops import _native; _native.native()" || { echo "native extension stale or missing"; exit 1; }
timeout -k 10 600 python -u -m pytest tests/test_conv_kernels.py -m gpu -x -v -p no:cacheprovider --timeout 200 --timeout-method thread -k "h3 or join_backward or celu_join" > "$OUT/pytest_h3.log" 2>&1; rc=$?
echo "pytest h3 rc=$rc"; tail -1 "$OUT/pytest_h3.log"
case $rc in 0) ;; 1) grep -E "^(FAILED|ERROR)|Error|assert" "$OUT/pytest_h3.log" | head -20; exit 1;; *) echo aborted; tail -20 "$OUT/pytest_h3.log"; exit 1;; esac
timeout -k 10 300 python -u scripts/bench_h3.py --batch 1024 > "$OUT/bench_h3_1024.txt" 2>&1 || { echo "bench_h3 failed"; tail -20 "$OUT/bench_h3_1024.txt"; exit 1; }
cat "$OUT/bench_h3_1024.txt" | grep -v amdgpu.ids
timeout -k 10 300 python -u scripts/bench_h3.py --batch 128 > "$OUT/bench_h3_128.txt" 2>&1 || { echo "bench_h3 128 failed"; exit 1; }
cat "$OUT/bench_h3_128.txt" | grep -v amdgpu.ids
timeout -k 10 600 python -u -m pytest tests/test_conv_kernels.py tests/test_resnet_engine.py -m gpu -x -v -p no:cacheprovider --timeout 200 --timeout-method thread > "$OUT/pytest.log" 2>&1; rc=$?
echo "pytest rc=$rc"; tail -1 "$OUT/pytest.log"
case $rc in 0) ;; 1) grep -E "^(FAILED|ERROR)" "$OUT/pytest.log" | head -20; exit 1;; *) echo aborted; tail -20 "$OUT/pytest.log"; exit 1;; esac
timeout -k 10 300 python bench.py > "$OUT/bench_default.log" 2>&1 || { echo "bench failed"; tail -5 "$OUT/bench_default.log"; exit 1; }
grep -h '"value"' "$OUT/bench_default.log" > "$OUT/bench_default.json"; grep -o '"ms_per_step": [0-9.]*' "$OUT/bench_default.json"
timeout -k 10 1200 python -u scripts/convergence_ablation.py --seeds 5 --out "$OUT/convergence_ablation.json" > "$OUT/convergence_ablation.txt" 2>&1 || { echo "ablation failed"; tail -20 "$OUT/convergence_ablation.txt"; exit 1; }
tail -20 "$OUT/convergence_ablation.txt"
