#!/usr/bin/env bash
# Round 4, fourth call: NGD R x R product kernels (micro-bench + step), NGD convergence with the
# fp64 fallback eigensolver, engine / FSDP / wgrad tests after the fixes, host profile of the
# transformer at 32 samples per GPU.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r4d}
mkdir -p "$OUT"
timeout -k 10 300 python scripts/bench_ngd.py --gemm-micro > "$OUT/ngd_gemm_micro.txt" 2>&1 && tail -1 "$OUT/ngd_gemm_micro.txt"
timeout -k 10 300 python scripts/bench_ngd.py > "$OUT/ngd_w1.txt" 2>&1 && tail -2 "$OUT/ngd_w1.txt"
timeout -k 10 300 python scripts/bench_ngd.py --world 8 > "$OUT/ngd_w8.txt" 2>&1 && tail -1 "$OUT/ngd_w8.txt"
timeout -k 10 600 python -u -m pytest tests/test_conv_kernels.py::test_conv_wgrad tests/test_resnet_engine.py \
  tests/test_distributed_gpu.py tests/test_gpu_kernels.py -k "wgrad or resnet_engine or fsdp_static or transformer_fsdp or ngd or mixup" \
  -m gpu -v -p no:cacheprovider --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1; rc=$?
echo "pytest rc=$rc"; tail -1 "$OUT/pytest.log"
case $rc in 0|1) ;; *) echo "pytest aborted rc=$rc"; exit 1;; esac
grep -E "^(FAILED|ERROR)" "$OUT/pytest.log" | head -20
timeout -k 10 400 python -u scripts/convergence.py --steps 300 --out "$OUT/convergence.json" > "$OUT/convergence.log" 2>&1 || { echo convergence failed; tail -5 "$OUT/convergence.log"; exit 1; }
tail -2 "$OUT/convergence.log"
timeout -k 10 300 python -u scripts/host_profile.py --model transformer --batch 32 --steps 40 > "$OUT/host_tr32.txt" 2>&1 && head -1 "$OUT/host_tr32.txt"
echo done
