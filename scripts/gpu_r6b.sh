#!/usr/bin/env bash
# Round 6: engine tests with the halo loop on, default bench, halo PMC passes, convergence ablation.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r6b}
mkdir -p "$OUT"
FDT_NATIVE=1 timeout -k 10 120 python -c "from faster_distributed_training_amd.ops import _native; _native.native()" || { echo "native extension stale or missing"; exit 1; }
timeout -k 10 300 python -u scripts/bench_h3.py --batch 1024 > "$OUT/bench_h3_1024.txt" 2>&1 || { echo "bench_h3 failed"; tail -20 "$OUT/bench_h3_1024.txt"; exit 1; }
grep -v amdgpu.ids "$OUT/bench_h3_1024.txt"
bash scripts/pmc_h3.sh "${1:-r6b}/pmc_h3" || exit 1
timeout -k 10 600 python -u -m pytest tests/test_resnet_engine.py tests/test_conv_kernels.py -m gpu -x -v -p no:cacheprovider --timeout 200 --timeout-method thread > "$OUT/pytest.log" 2>&1; rc=$?
echo "pytest rc=$rc"; tail -1 "$OUT/pytest.log"
case $rc in 0) ;; 1) grep -E "^(FAILED|ERROR)|^E " "$OUT/pytest.log" | head -20; exit 1;; *) echo aborted; tail -20 "$OUT/pytest.log"; exit 1;; esac
timeout -k 10 300 python bench.py > "$OUT/bench_default.log" 2>&1 || { echo "bench failed"; tail -5 "$OUT/bench_default.log"; exit 1; }
grep -h '"value"' "$OUT/bench_default.log" > "$OUT/bench_default.json"; grep -o '"ms_per_step": [0-9.]*' "$OUT/bench_default.json"
FDT_CONV_H3=0 timeout -k 10 300 python bench.py > "$OUT/bench_noh3.log" 2>&1 || { echo "bench noh3 failed"; exit 1; }
grep -h '"value"' "$OUT/bench_noh3.log" > "$OUT/bench_noh3.json"; grep -o '"ms_per_step": [0-9.]*' "$OUT/bench_noh3.json"
timeout -k 10 1200 python -u scripts/convergence_ablation.py --seeds 5 --out "$OUT/convergence_ablation.json" > "$OUT/convergence_ablation.txt" 2>&1 || { echo "ablation failed"; tail -20 "$OUT/convergence_ablation.txt"; exit 1; }
tail -20 "$OUT/convergence_ablation.txt"
