#!/usr/bin/env bash
# Round 4: Jacobi with the transposed float4 eigenvector accumulator -- tests, timing, benches.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r4q}
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_ngd_graphs.py -k "eigh or ngd" -m gpu -v -p no:cacheprovider \
  --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1; rc=$?
echo "pytest rc=$rc"; tail -1 "$OUT/pytest.log"
case $rc in 0) ;; 1) grep -E "^(FAILED|ERROR)|Error" "$OUT/pytest.log" | head -30; exit 1;; *) echo aborted; exit 1;; esac
timeout -k 10 300 python -u scripts/probe_eigh_sweeps.py > "$OUT/eigh_sweeps.txt" 2>&1 && grep sweeps "$OUT/eigh_sweeps.txt" | head -4 || exit 1
run() {
  local name=$1; shift
  timeout -k 10 300 python bench.py "$@" > "$OUT/$name.log" 2>&1 || { echo "$name failed"; tail -5 "$OUT/$name.log"; exit 1; }
  grep -h '"value"' "$OUT/$name.log" > "$OUT/$name.json"
  echo "$name $(grep -o '"ms_per_step": [0-9.]*' "$OUT/$name.json")"
}
run tr_b32 --model transformer --global-batch 32 --steps 40 --warmup 12
run tr_b256 --model transformer --steps 20 --warmup 12
run ngd_meta --ngd --meta_learning --steps 20 --warmup 12
timeout -k 10 300 python scripts/bench_ngd.py --world 8 --graphs > "$OUT/ngd_w8_graphs.txt" 2>&1 && tail -1 "$OUT/ngd_w8_graphs.txt" || exit 1
timeout -k 10 300 python scripts/bench_ngd.py > "$OUT/ngd_w1.txt" 2>&1 && tail -2 "$OUT/ngd_w1.txt" || exit 1
echo done
