#!/usr/bin/env bash
# Round 4: Jacobi eigh round loop (upper-triangle A, no divisions in the round), LayerNorm
# backward grid / prefetch -- tests, eigh sweep timing on the transformer's matrices, benches.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r4j}
mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_transformer_graphs.py -k "eigh or layernorm or ngd or transformer" -m gpu -v -p no:cacheprovider \
  --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1; rc=$?
echo "pytest rc=$rc"; tail -1 "$OUT/pytest.log"
case $rc in 0) ;; 1) grep -E "^(FAILED|ERROR)|Error" "$OUT/pytest.log" | head -30; exit 1;; *) echo aborted; exit 1;; esac
timeout -k 10 300 python -u scripts/probe_eigh_sweeps.py > "$OUT/eigh_sweeps.txt" 2>&1 && grep sweeps "$OUT/eigh_sweeps.txt" | head -3 || exit 1
run() {
  local name=$1; shift
  timeout -k 10 300 python bench.py "$@" > "$OUT/$name.log" 2>&1 || { echo "$name failed"; tail -5 "$OUT/$name.log"; exit 1; }
  grep -h '"value"' "$OUT/$name.log" > "$OUT/$name.json"
  echo "$name $(grep -o '"ms_per_step": [0-9.]*' "$OUT/$name.json") $(grep -o '"host_ms_per_step": [0-9.]*' "$OUT/$name.json")"
}
run tr_b32 --model transformer --global-batch 32 --steps 40 --warmup 12
run tr_b256 --model transformer --steps 20 --warmup 12
timeout -k 10 300 python scripts/bench_ngd.py > "$OUT/ngd_w1.txt" 2>&1 && tail -2 "$OUT/ngd_w1.txt" || exit 1
timeout -k 10 300 python scripts/bench_ngd.py --world 8 > "$OUT/ngd_w8.txt" 2>&1 && tail -1 "$OUT/ngd_w8.txt" || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_b32" -o run -- python bench.py --model transformer --global-batch 32 --steps 30 --warmup 10 > "$OUT/prof_b32.log" 2>&1 || { echo prof failed; exit 1; }
f=$(find "$OUT/prof_b32" -name '*kernel_stats.csv' | head -n 1)
python scripts/kstats.py "$f" --steps 40 --top 45 > "$OUT/kstats_tr_b32.txt"; head -8 "$OUT/kstats_tr_b32.txt"
echo done
