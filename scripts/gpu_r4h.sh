#!/usr/bin/env bash
# Round 4: NGD projection on the matrix cores (v_mfma_f32_16x16x4_f32) -- bitwise parity with
# the VALU form, then A/B on the NGD step bench and the transformer at 32 / 256 samples.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r4h}
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k "ngd" -m gpu -v -p no:cacheprovider \
  --timeout 120 --timeout-method thread > "$OUT/pytest_ngd.log" 2>&1; rc=$?
echo "pytest ngd rc=$rc"; tail -1 "$OUT/pytest_ngd.log"
case $rc in 0) ;; 1) grep -E "^(FAILED|ERROR)|assert|Error" "$OUT/pytest_ngd.log" | head -30; exit 1;; *) echo aborted; exit 1;; esac
timeout -k 10 300 python scripts/bench_ngd.py > "$OUT/ngd_w1_mfma.txt" 2>&1 && tail -2 "$OUT/ngd_w1_mfma.txt" || exit 1
FDT_NGD_MFMA=0 timeout -k 10 300 python scripts/bench_ngd.py > "$OUT/ngd_w1_valu.txt" 2>&1 && tail -2 "$OUT/ngd_w1_valu.txt" || exit 1
run() {
  local name=$1; shift
  timeout -k 10 300 python bench.py "$@" > "$OUT/$name.log" 2>&1 || { echo "$name failed"; tail -5 "$OUT/$name.log"; exit 1; }
  grep -h '"value"' "$OUT/$name.log" > "$OUT/$name.json"
  echo "$name $(grep -o '"ms_per_step": [0-9.]*' "$OUT/$name.json") $(grep -o '"host_ms_per_step": [0-9.]*' "$OUT/$name.json")"
}
run tr_b32_mfma --model transformer --global-batch 32 --steps 40 --warmup 12
FDT_NGD_MFMA=0 run tr_b32_valu --model transformer --global-batch 32 --steps 40 --warmup 12
run tr_b256_mfma --model transformer --steps 20 --warmup 12
FDT_NGD_MFMA=0 run tr_b256_valu --model transformer --steps 20 --warmup 12
run ngd_meta_mfma --ngd --meta_learning --steps 20 --warmup 12
FDT_NGD_MFMA=0 run ngd_meta_valu --ngd --meta_learning --steps 20 --warmup 12
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_b32" -o run -- python bench.py --model transformer --global-batch 32 --steps 30 --warmup 10 > "$OUT/prof_b32.log" 2>&1 || { echo prof failed; exit 1; }
f=$(find "$OUT/prof_b32" -name '*kernel_stats.csv' | head -n 1)
python scripts/kstats.py "$f" --steps 40 --top 45 > "$OUT/kstats_tr_b32_mfma.txt"; head -12 "$OUT/kstats_tr_b32_mfma.txt"
echo done
