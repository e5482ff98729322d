#!/usr/bin/env bash
# Round 4, fifth call: the LDS-DMA 3-buffer ring (kg=3) for the prologue-free convolutions --
# bitwise parity with the register-staged path, engine parity with it switched on, and A/B
# at the two batch sizes plus per-layer rooflines (engine variants); NGD W-update micro.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r4e}
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest tests/test_conv_kernels.py -k "lds_dma_ring" -m gpu -v -p no:cacheprovider \
  --timeout 120 --timeout-method thread > "$OUT/pytest_glds.log" 2>&1; rc=$?
echo "pytest glds rc=$rc"; tail -1 "$OUT/pytest_glds.log"
case $rc in 0) ;; 1) grep -E "^(FAILED|ERROR)|Error" "$OUT/pytest_glds.log" | head -20; exit 1;; *) echo "aborted"; exit 1;; esac
FDT_CONV_GLDS=1 timeout -k 10 400 python -u -m pytest tests/test_resnet_engine.py -m gpu -v -p no:cacheprovider \
  --timeout 200 --timeout-method thread > "$OUT/pytest_engine_glds.log" 2>&1; rc=$?
echo "pytest engine(glds) rc=$rc"; tail -1 "$OUT/pytest_engine_glds.log"
case $rc in 0|1) ;; *) echo "aborted"; exit 1;; esac
grep -E "^(FAILED|ERROR)" "$OUT/pytest_engine_glds.log" | head -20
run() {
  local name=$1; shift
  timeout -k 10 300 python bench.py "$@" > "$OUT/$name.log" 2>&1 || { echo "$name failed"; tail -5 "$OUT/$name.log"; exit 1; }
  grep -h '"value"' "$OUT/$name.log" > "$OUT/$name.json"
  echo "$name $(grep -o '"ms_per_step": [0-9.]*' "$OUT/$name.json")"
}
run bs128 --steps 40 --warmup 5 --global-batch 128
FDT_CONV_GLDS=1 run bs128_glds --steps 40 --warmup 5 --global-batch 128
run bs1024 --steps 30 --warmup 5
FDT_CONV_GLDS=1 run bs1024_glds --steps 30 --warmup 5
mkdir -p "$OUT/pmc"
for b in 128 1024; do
  timeout -k 10 300 python scripts/roofline_layers.py --batch $b --md "$OUT/pmc/roof$b.md" --json "$OUT/pmc/roof$b.json" > "$OUT/roof$b.log" 2>&1 && tail -1 "$OUT/roof$b.log" || exit 1
  FDT_CONV_GLDS=1 timeout -k 10 300 python scripts/roofline_layers.py --batch $b --md "$OUT/pmc/roof${b}_glds.md" --json "$OUT/pmc/roof${b}_glds.json" > "$OUT/roof${b}_glds.log" 2>&1 && tail -1 "$OUT/roof${b}_glds.log" || exit 1
done
timeout -k 10 300 python scripts/bench_ngd.py --gemm-micro > "$OUT/ngd_gemm_micro.txt" 2>&1 && tail -2 "$OUT/ngd_gemm_micro.txt"
echo done
