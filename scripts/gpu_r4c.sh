#!/usr/bin/env bash
# Round 4, A/B call: join fold width at bs1024 / bs128, NGD graph replay for the transformer
# and the ResNet NGD+meta path, sharded NGD at world 1.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r4c}
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests/test_conv_kernels.py::test_conv_wgrad "tests/test_resnet_engine.py::test_engine_train_step_matches_reference" \
  tests/test_distributed_gpu.py -k "wgrad or matches_reference or fsdp_static or transformer_fsdp" -m gpu -v -p no:cacheprovider \
  --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1; rc=$?
echo "pytest rc=$rc"; tail -1 "$OUT/pytest.log"
case $rc in 0|1) ;; *) echo "pytest aborted rc=$rc"; exit 1;; esac
grep -E "^(FAILED|ERROR)" "$OUT/pytest.log" | head -20
timeout -k 10 400 python -u scripts/convergence.py --steps 300 --out "$OUT/convergence.json" > "$OUT/convergence.log" 2>&1 || { echo convergence failed; tail -5 "$OUT/convergence.log"; exit 1; }
tail -2 "$OUT/convergence.log"
run() {
  local name=$1; shift
  timeout -k 10 300 python bench.py "$@" > "$OUT/$name.log" 2>&1 || { echo "$name failed"; tail -5 "$OUT/$name.log"; exit 1; }
  grep -h '"value"' "$OUT/$name.log" > "$OUT/$name.json"
  echo "$name $(grep -o '"ms_per_step": [0-9.]*' "$OUT/$name.json") $(grep -o '"host_ms_per_step": [0-9.]*' "$OUT/$name.json")"
}
run bs1024_fold64 --steps 30 --warmup 5
FDT_JOIN_FOLD_MAX=128 run bs1024_fold128 --steps 30 --warmup 5
FDT_JOIN_FOLD_MAX=256 run bs1024_fold256 --steps 30 --warmup 5
run bs1024_fold64b --steps 30 --warmup 5
FDT_JOIN_FOLD_MAX=128 run bs128_fold128 --steps 40 --warmup 5 --global-batch 128
FDT_JOIN_FOLD_MAX=256 run bs128_fold256 --steps 40 --warmup 5 --global-batch 128
run bs128_fold64 --steps 40 --warmup 5 --global-batch 128
FDT_WG_STAGES=4 run bs128_wg4 --steps 40 --warmup 5 --global-batch 128
FDT_WG_STAGES=4 run bs1024_wg4 --steps 30 --warmup 5
FDT_WG_FUSED_REDUCE=1 run bs128_wgfr --steps 40 --warmup 5 --global-batch 128
FDT_WG_FUSED_REDUCE=1 FDT_WG_STAGES=4 run bs128_wgfr4 --steps 40 --warmup 5 --global-batch 128
FDT_WG_FUSED_REDUCE=1 run bs1024_wgfr --steps 30 --warmup 5
run tr_b32 --model transformer --global-batch 32 --steps 40 --warmup 12
FDT_NGD_GRAPHS=1 run tr_b32_ngdg --model transformer --global-batch 32 --steps 40 --warmup 12
FDT_NGD_GRAPHS=1 run tr_b256_ngdg --model transformer --steps 20 --warmup 12
run ngd_meta --ngd --meta_learning --steps 20 --warmup 12
FDT_NGD_GRAPHS=1 run ngd_meta_ngdg --ngd --meta_learning --steps 20 --warmup 12
FDT_NGD_GEMM=0 run ngd_meta_libgemm --ngd --meta_learning --steps 20 --warmup 12
run ngd_meta_sharded --ngd --meta_learning --sharded-ngd --steps 20 --warmup 12

mkdir -p "$OUT/pmc"
timeout -k 10 300 python scripts/roofline_layers.py --batch 1024 --md "$OUT/pmc/r4_bs1024_roofline.md" > "$OUT/roof1024.log" 2>&1 && tail -1 "$OUT/roof1024.log"
timeout -k 10 300 python scripts/roofline_layers.py --batch 128 --md "$OUT/pmc/r4_bs128_roofline.md" > "$OUT/roof128.log" 2>&1 && tail -1 "$OUT/roof128.log"
FDT_NGD_GEMM=0 timeout -k 10 300 python scripts/bench_ngd.py --world 8 > "$OUT/ngd_w8_libgemm.txt" 2>&1 && tail -1 "$OUT/ngd_w8_libgemm.txt"
timeout -k 10 300 python scripts/bench_ngd.py > "$OUT/ngd_w1.txt" 2>&1 && tail -2 "$OUT/ngd_w1.txt"
FDT_NGD_GEMM=0 timeout -k 10 300 python scripts/bench_ngd.py > "$OUT/ngd_w1_libgemm.txt" 2>&1 && tail -2 "$OUT/ngd_w1_libgemm.txt"
echo done
