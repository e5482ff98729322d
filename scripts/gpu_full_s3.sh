#!/usr/bin/env bash
# Full GPU evidence (round 3, session 3): every -m gpu test, smoke, default bench, the BASELINE
# configs on one GPU, and a kernel profile of the default bench.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${1:-full_s3b}
mkdir -p "$OUT"
timeout -k 10 900 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1; rc=$?
echo "pytest rc=$rc" >> "$OUT/pytest.log"; tail -3 "$OUT/pytest.log"
case $rc in 0|1) ;; *) echo "pytest aborted rc=$rc"; exit 1;; esac
grep -E "^(FAILED|ERROR)" "$OUT/pytest.log" | head -20
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { echo smoke failed; tail "$OUT/smoke.log"; exit 1; }
tail -1 "$OUT/smoke.log"
run() {  # name, args...
  local name=$1; shift
  timeout -k 10 300 python bench.py "$@" > "$OUT/$name.log" 2>&1 || { echo "$name failed"; tail -5 "$OUT/$name.log"; exit 1; }
  grep -h '"value"' "$OUT/$name.log" > "$OUT/$name.json"
  echo "$name $(grep -o '"ms_per_step": [0-9.]*' "$OUT/$name.json")"
}
run default
run bs1024 --steps 30 --warmup 5
run bs128 --steps 40 --warmup 5 --global-batch 128
run ngd_meta --ngd --meta_learning --steps 20 --warmup 12
run fsdp --fsdp --steps 10 --warmup 3
run transformer --model transformer --steps 20 --warmup 12
run transformer_b32 --model transformer --global-batch 32 --steps 40 --warmup 12
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- python bench.py --steps 4 --warmup 3 > "$OUT/prof.log" 2>&1 || { echo prof failed; exit 1; }
f=$(find "$OUT/prof" -name '*kernel_stats.csv' | head -n 1)
python scripts/kstats.py "$f" --steps 7 --top 50 > "$OUT/kstats_bs1024.txt"
echo done
