#!/usr/bin/env bash
# Round 5 closing measurements: whole GPU suite + smoke, headline / 8-GPU-share / DDP benches,
# transformer, FSDP offload, world-8 sharded NGD simulation, NGD meta-mixup dp1 vs sharded,
# convergence curves.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r5z}
mkdir -p "$OUT"
FDT_NATIVE=1 timeout -k 10 120 python -c "from faster_distributed_training_amd.ops import _native; _native.native()" || { echo "native extension stale or missing"; exit 1; }
timeout -k 10 1500 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 400 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1; rc=$?
echo "pytest rc=$rc"; tail -1 "$OUT/pytest_gpu.log"
case $rc in 0) ;; 1) grep -E "^(FAILED|ERROR)" "$OUT/pytest_gpu.log" | head -20;; *) echo aborted; tail -20 "$OUT/pytest_gpu.log"; exit 1;; esac
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 && tail -1 "$OUT/smoke.log" || { echo smoke failed; tail -5 "$OUT/smoke.log"; exit 1; }
run() {
  local name=$1; shift
  timeout -k 10 300 python bench.py "$@" > "$OUT/$name.log" 2>&1 || { echo "$name failed"; tail -5 "$OUT/$name.log"; exit 1; }
  grep -h '"value"' "$OUT/$name.log" > "$OUT/$name.json"
  echo "$name $(grep -o '"ms_per_step": [0-9.]*' "$OUT/$name.json") $(grep -o '"graph_comm": "[^"]*"' "$OUT/$name.json")"
}
run bench_default
run bs1024 --steps 30 --warmup 8
run bs128 --steps 40 --warmup 5 --global-batch 128
run bs128_ddp --steps 40 --warmup 5 --global-batch 128 --ddp
run tr_b256 --model transformer --steps 20 --warmup 12
run tr_b32 --model transformer --global-batch 32 --steps 40 --warmup 12
run tr_fsdp_offload --model transformer --fsdp --fsdp-offload --steps 10 --warmup 4
run ngd_meta --ngd --meta_learning --steps 20 --warmup 12
run ngd_meta_sharded --ngd --meta_learning --sharded-ngd --steps 20 --warmup 12
for m in transformer resnet50; do
  timeout -k 10 300 python scripts/bench_ngd.py --model $m --world 8 --graphs > "$OUT/ngd_w8_${m}_graphs.txt" 2>&1 || { echo "ngd w8 $m failed"; exit 1; }
  tail -1 "$OUT/ngd_w8_${m}_graphs.txt"
done
timeout -k 10 600 python scripts/convergence.py --opts madgrad,ngd --arch resnet18 --out "$OUT/convergence_resnet18.json" > "$OUT/convergence_resnet18.log" 2>&1 && tail -2 "$OUT/convergence_resnet18.log" || { echo "convergence r18 failed"; exit 1; }
timeout -k 10 600 python scripts/convergence.py --opts madgrad --arch resnet50 --out "$OUT/convergence_resnet50.json" > "$OUT/convergence_resnet50.log" 2>&1 && tail -2 "$OUT/convergence_resnet50.log" || { echo "convergence r50 failed"; exit 1; }
echo done
