#!/usr/bin/env bash
# Round 4: single-rank all-reduce / reduce-scatter as SUM (no PreMulSum pass) -- RCCL world-1
# tests, DDP / FSDP / sharded-NGD benches, kernel list of the DDP proxy.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r4aa}
mkdir -p "$OUT"
timeout -k 10 700 python -u -m pytest tests/test_distributed_gpu.py -m gpu -v -p no:cacheprovider --timeout 650 --timeout-method thread > "$OUT/pytest.log" 2>&1; rc=$?
echo "pytest rc=$rc"; tail -1 "$OUT/pytest.log"
case $rc in 0) ;; 1) grep -E "^(FAILED|ERROR)" "$OUT/pytest.log" | head -20; exit 1;; *) echo aborted; exit 1;; esac
run() {
  local name=$1; shift
  timeout -k 10 300 python bench.py "$@" > "$OUT/$name.log" 2>&1 || { echo "$name failed"; tail -5 "$OUT/$name.log"; exit 1; }
  grep -h '"value"' "$OUT/$name.log" > "$OUT/$name.json"
  echo "$name $(grep -o '"ms_per_step": [0-9.]*' "$OUT/$name.json")"
}
run bs128 --steps 40 --warmup 5 --global-batch 128
run bs128_ddp --steps 40 --warmup 5 --global-batch 128 --ddp
run bs1024 --steps 30 --warmup 8
run bs1024_ddp --steps 30 --warmup 8 --ddp
run fsdp_full --fsdp --steps 20 --warmup 8
run ngd_meta_sharded --ngd --meta_learning --sharded-ngd --steps 20 --warmup 12
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_ddp" -o run -- python bench.py --global-batch 128 --steps 30 --warmup 5 --ddp > "$OUT/prof_ddp.log" 2>&1 || { echo prof failed; exit 1; }
f=$(find "$OUT/prof_ddp" -name '*kernel_stats.csv' | head -n 1)
python scripts/kstats.py "$f" --steps 35 --top 80 > "$OUT/kstats_bs128_ddp.txt"; grep -i "oneRank\|fillBuffer\|copyBuffer" "$OUT/kstats_bs128_ddp.txt" || true
echo done
