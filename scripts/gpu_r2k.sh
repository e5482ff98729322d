#!/usr/bin/env bash
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r2k}
mkdir -p "$OUT"
timeout -k 10 500 python -u -m pytest tests/test_attention_gpu.py tests/test_transformer_graphs.py tests/test_distributed_gpu.py -m gpu -v -p no:cacheprovider --timeout 200 --timeout-method thread > "$OUT/pytest.log" 2>&1; rc=$?; echo "pytest rc=$rc" >> "$OUT/pytest.log"
case $rc in 0|1) ;; *) echo "pytest aborted rc=$rc"; exit 1;; esac
timeout -k 10 300 python bench.py --model transformer --steps 20 --warmup 12 > "$OUT/bench_tr.log" 2>&1 || { echo bench_tr failed; exit 1; }
timeout -k 10 300 python bench.py --model transformer --steps 20 --warmup 12 --seq-buckets 128,192 > "$OUT/bench_tr192.log" 2>&1 || { echo bench_tr192 failed; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_tr" -o run -- python3 bench.py --model transformer --steps 10 --warmup 12 --seq-buckets 256 > "$OUT/prof_tr.log" 2>&1 || { echo prof failed; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof1024" -o run -- python3 bench.py --steps 5 --warmup 3 > "$OUT/prof1024.log" 2>&1 || { echo prof1024 failed; exit 1; }
echo done
