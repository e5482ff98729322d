#!/usr/bin/env bash
# Round 6: per-rank world-8 steps on one GPU (bench.py --simulate-world 8) for the BASELINE
# configs + transformer host profiles at the 8-GPU share (B=32) and B=256.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r6c}
NGD_RANKS=${NGD_RANKS:-"0 1 2 3 4 5 6 7"}
mkdir -p "$OUT"
FDT_NATIVE=1 timeout -k 10 120 python -c "from faster_distributed_training_amd.ops import _native; _native.native()" || { echo "native extension stale or missing"; exit 1; }
timeout -k 10 300 python bench.py > "$OUT/bench_default.log" 2>&1 || { echo "bench failed"; tail -5 "$OUT/bench_default.log"; exit 1; }
grep -h '"value"' "$OUT/bench_default.log" > "$OUT/bench_default.json"; echo "bs1024 $(grep -o '"ms_per_step": [0-9.]*' $OUT/bench_default.json)"
timeout -k 10 300 python bench.py --global-batch 128 --steps 40 > "$OUT/bs128.log" 2>&1 || { echo "bs128 failed"; exit 1; }
grep -h '"value"' "$OUT/bs128.log" > "$OUT/bs128.json"; echo "bs128 $(grep -o '"ms_per_step": [0-9.]*' $OUT/bs128.json)"
timeout -k 10 900 python -u -m pytest tests/test_simulate.py tests/test_distributed_gpu.py -m gpu -x -v -p no:cacheprovider --timeout 600 --timeout-method thread -k "offload or simulated" > "$OUT/pytest_new.log" 2>&1; rc=$?
echo "pytest new rc=$rc"; tail -1 "$OUT/pytest_new.log"
case $rc in 0) ;; 1) grep -E "^(FAILED|ERROR)|^E " "$OUT/pytest_new.log" | head -20;; *) echo aborted; tail -20 "$OUT/pytest_new.log"; exit 1;; esac
for r in $NGD_RANKS; do
  timeout -k 10 300 python bench.py --ngd --meta_learning --simulate-world 8 --simulate-rank $r --steps 20 --warmup 12 > "$OUT/sim_ngd_meta_r$r.log" 2>&1 || { echo "sim ngd_meta r$r failed"; tail -5 "$OUT/sim_ngd_meta_r$r.log"; exit 1; }
  grep -h '"value"' "$OUT/sim_ngd_meta_r$r.log" > "$OUT/sim_ngd_meta_r$r.json"; echo "ngd_meta r$r $(grep -o '"ms_per_step": [0-9.]*' $OUT/sim_ngd_meta_r$r.json) $(grep -o '"host_ms_per_step": [0-9.]*' $OUT/sim_ngd_meta_r$r.json)"
done
for r in 0 7; do
  timeout -k 10 300 python bench.py --simulate-world 8 --simulate-rank $r --steps 20 --warmup 8 > "$OUT/sim_ddp_r$r.log" 2>&1 || { echo "sim ddp r$r failed"; tail -5 "$OUT/sim_ddp_r$r.log"; exit 1; }
  grep -h '"value"' "$OUT/sim_ddp_r$r.log" > "$OUT/sim_ddp_r$r.json"; echo "ddp r$r $(grep -o '"ms_per_step": [0-9.]*' $OUT/sim_ddp_r$r.json) $(grep -o '"host_ms_per_step": [0-9.]*' $OUT/sim_ddp_r$r.json)"
  timeout -k 10 300 python bench.py --fsdp --simulate-world 8 --simulate-rank $r --steps 20 --warmup 8 > "$OUT/sim_fsdp_r$r.log" 2>&1 || { echo "sim fsdp r$r failed"; tail -5 "$OUT/sim_fsdp_r$r.log"; exit 1; }
  grep -h '"value"' "$OUT/sim_fsdp_r$r.log" > "$OUT/sim_fsdp_r$r.json"; echo "fsdp r$r $(grep -o '"ms_per_step": [0-9.]*' $OUT/sim_fsdp_r$r.json) $(grep -o '"host_ms_per_step": [0-9.]*' $OUT/sim_fsdp_r$r.json)"
  timeout -k 10 300 python bench.py --model transformer --simulate-world 8 --simulate-rank $r --steps 30 --warmup 15 > "$OUT/sim_tr_r$r.log" 2>&1 || { echo "sim tr r$r failed"; tail -5 "$OUT/sim_tr_r$r.log"; exit 1; }
  grep -h '"value"' "$OUT/sim_tr_r$r.log" > "$OUT/sim_tr_r$r.json"; echo "tr r$r $(grep -o '"ms_per_step": [0-9.]*' $OUT/sim_tr_r$r.json) $(grep -o '"host_ms_per_step": [0-9.]*' $OUT/sim_tr_r$r.json)"
done
for o in device host; do
  timeout -k 10 900 python bench.py --model transformer --fsdp --fsdp-offload --fsdp-offload-optimizer $o --steps 10 --warmup 4 > "$OUT/tr_fsdp_offload_$o.log" 2>&1 || { echo "offload $o failed"; tail -5 "$OUT/tr_fsdp_offload_$o.log"; exit 1; }
  grep -h '"value"' "$OUT/tr_fsdp_offload_$o.log" > "$OUT/tr_fsdp_offload_$o.json"; echo "tr fsdp offload $o $(grep -o '"ms_per_step": [0-9.]*' $OUT/tr_fsdp_offload_$o.json)"
done
timeout -k 10 300 python bench.py --fsdp --steps 20 --warmup 8 > "$OUT/r50_fsdp.log" 2>&1 || { echo "r50 fsdp failed"; exit 1; }
grep -h '"value"' "$OUT/r50_fsdp.log" > "$OUT/r50_fsdp.json"; echo "r50 fsdp bs1024 $(grep -o '"ms_per_step": [0-9.]*' $OUT/r50_fsdp.json)"
for b in 32 256; do
  timeout -k 10 300 python scripts/host_profile_tr.py --batch $b --steps 20 > "$OUT/host_tr_b$b.txt" 2>&1 || { echo "host profile b$b failed"; tail -5 "$OUT/host_tr_b$b.txt"; exit 1; }
done
echo done
