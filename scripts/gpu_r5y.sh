#!/usr/bin/env bash
# Transformer step glue: adjacent Q/K/V shadows (no per-forward concat), one mask cast, mixup_prep
# + fused meter in the replayed step.  Transformer GPU tests + B=32 / B=256 benches.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r5y}
mkdir -p "$OUT"
FDT_NATIVE=1 timeout -k 10 120 python -c "from faster_distributed_training_amd.ops import _native; _native.native()" || { echo "native extension stale or missing"; exit 1; }
timeout -k 10 900 python -u -m pytest tests/test_transformer_graphs.py tests/test_transformer_fusions.py tests/test_attention_gpu.py tests/test_linear.py tests/test_ngd_graphs.py tests/test_gpu_kernels.py -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1; rc=$?
echo "pytest rc=$rc"; tail -1 "$OUT/pytest.log"; grep -E "^(FAILED|ERROR)" "$OUT/pytest.log" | head; case $rc in 0|1) ;; *) exit 1;; esac
run() {
  local name=$1; shift
  timeout -k 10 300 python bench.py "$@" > "$OUT/$name.log" 2>&1 || { echo "$name failed"; tail -5 "$OUT/$name.log"; exit 1; }
  grep -h '"value"' "$OUT/$name.log" > "$OUT/$name.json"
  echo "$name $(grep -o '"ms_per_step": [0-9.]*' "$OUT/$name.json") $(grep -o '"host_ms_per_step": [0-9.]*' "$OUT/$name.json")"
}
run tr_b32_a --model transformer --global-batch 32 --steps 40 --warmup 12
run tr_b32_b --model transformer --global-batch 32 --steps 40 --warmup 12
run tr_b256 --model transformer --steps 20 --warmup 12
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_tr_b32" -o run -- python3 bench.py --model transformer --global-batch 32 --steps 12 --warmup 12 > "$OUT/prof_tr_b32.log" 2>&1 || { echo "prof failed"; tail -5 "$OUT/prof_tr_b32.log"; exit 1; }
f=$(find "$OUT/prof_tr_b32" -name '*kernel_stats.csv' | head -n 1)
python scripts/kstats.py "$f" --steps 24 --top 50 > "$OUT/kstats_tr_b32.txt"
head -2 "$OUT/kstats_tr_b32.txt"
echo done
