#!/usr/bin/env bash
# Round 6 closing run on the final tree: the GPU test suite + smoke, the headline / 8-GPU-share
# benches, the world-8 rank rehearsals with host busy time, FSDP + offload, and kernel traces.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r6z}
MODE=${MODE:-bench}  # tests | bench
mkdir -p "$OUT"
FDT_NATIVE=1 timeout -k 10 120 python -c "from faster_distributed_training_amd.ops import _native; _native.native()" || { echo "native extension stale or missing"; exit 1; }
j() { grep -h '"value"' "$OUT/$1.log" > "$OUT/$1.json"; echo "$1 $(grep -o '"ms_per_step": [0-9.]*' $OUT/$1.json) $(grep -o '"host_ms_per_step": [0-9.]*' $OUT/$1.json) $(grep -o '"host_busy_ms_per_step": [0-9.]*' $OUT/$1.json)"; }
if [ "$MODE" = tests ]; then
  timeout -k 10 1080 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1; rc=$?
  echo "pytest gpu rc=$rc"; tail -1 "$OUT/pytest_gpu.log"
  case $rc in 0) ;; 1) grep -E "^(FAILED|ERROR)" "$OUT/pytest_gpu.log" | head -20;; *) echo aborted; tail -20 "$OUT/pytest_gpu.log"; exit 1;; esac
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$OUT/smoke.log" 2>&1 || { echo "smoke failed"; tail -5 "$OUT/smoke.log"; exit 1; }
  tail -1 "$OUT/smoke.log"
  exit 0
fi
timeout -k 10 300 python bench.py > "$OUT/bench_default.log" 2>&1 || { echo "bench failed"; tail -5 "$OUT/bench_default.log"; exit 1; }
j bench_default
timeout -k 10 300 python bench.py --global-batch 128 --steps 40 > "$OUT/bs128.log" 2>&1 || { echo "bs128 failed"; exit 1; }
j bs128
timeout -k 10 300 python bench.py --global-batch 128 --steps 40 --ddp > "$OUT/bs128_ddp.log" 2>&1 || { echo "bs128 ddp failed"; exit 1; }
j bs128_ddp
timeout -k 10 300 python bench.py --model transformer > "$OUT/tr_b256.log" 2>&1 || { echo "tr failed"; exit 1; }
j tr_b256
timeout -k 10 300 python bench.py --model transformer --global-batch 32 --steps 40 --warmup 15 > "$OUT/tr_b32.log" 2>&1 || { echo "tr b32 failed"; exit 1; }
j tr_b32
for r in 0 7; do
  timeout -k 10 300 python bench.py --model transformer --simulate-world 8 --simulate-rank $r --steps 30 --warmup 15 > "$OUT/sim_tr_r$r.log" 2>&1 || { echo "sim tr failed"; exit 1; }
  j sim_tr_r$r
done
for r in 6 7; do
  timeout -k 10 300 python bench.py --ngd --meta_learning --simulate-world 8 --simulate-rank $r --steps 20 --warmup 12 > "$OUT/sim_ngd_meta_r$r.log" 2>&1 || { echo "sim ngd failed"; exit 1; }
  j sim_ngd_meta_r$r
done
timeout -k 10 300 python bench.py --ngd --meta_learning --steps 20 --warmup 12 > "$OUT/ngd_meta.log" 2>&1 || { echo "ngd_meta failed"; exit 1; }
j ngd_meta
timeout -k 10 300 python bench.py --fsdp --steps 20 --warmup 8 > "$OUT/r50_fsdp.log" 2>&1 || { echo "r50 fsdp failed"; exit 1; }
j r50_fsdp
timeout -k 10 600 python bench.py --model transformer --fsdp --fsdp-offload --steps 10 --warmup 4 > "$OUT/tr_fsdp_offload.log" 2>&1 || { echo "offload failed"; exit 1; }
j tr_fsdp_offload
for b in 128 1024; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/kt_bs$b" -o kt -- python bench.py --global-batch $b --steps 15 --warmup 8 > "$OUT/kt_bs$b.log" 2>&1 || { echo "trace bs$b failed"; tail -5 "$OUT/kt_bs$b.log"; exit 1; }
  f=$(find "$OUT/kt_bs$b" -name '*kernel_stats.csv' | head -n 1); python scripts/kstats.py "$f" --steps 23 --top 60 > "$OUT/kstats_bs$b.txt"; head -1 "$OUT/kstats_bs$b.txt"
done
echo done
