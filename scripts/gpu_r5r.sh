#!/usr/bin/env bash
# Transformer at the 8-GPU share: B=32 step + kernel profile, world-8 sharded NGD (graphs / eager).
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r5r}
mkdir -p "$OUT"
FDT_NATIVE=1 timeout -k 10 120 python -c "from faster_distributed_training_amd.ops import _native; _native.native()" || { echo "native extension stale or missing"; exit 1; }
timeout -k 10 300 python bench.py --model transformer --global-batch 32 --steps 40 --warmup 12 > "$OUT/tr_b32.log" 2>&1 || { echo "b32 failed"; tail -5 "$OUT/tr_b32.log"; exit 1; }
grep -h '"value"' "$OUT/tr_b32.log" > "$OUT/tr_b32.json"; grep -o '"ms_per_step": [0-9.]*' "$OUT/tr_b32.json"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_tr_b32" -o run -- python3 bench.py --model transformer --global-batch 32 --steps 12 --warmup 12 > "$OUT/prof_tr_b32.log" 2>&1 || { echo "prof failed"; tail -5 "$OUT/prof_tr_b32.log"; exit 1; }
f=$(find "$OUT/prof_tr_b32" -name '*kernel_stats.csv' | head -n 1)
python scripts/kstats.py "$f" --steps 24 --top 50 > "$OUT/kstats_tr_b32.txt"
head -25 "$OUT/kstats_tr_b32.txt"
timeout -k 10 300 python scripts/bench_ngd.py --model transformer --world 8 --graphs > "$OUT/ngd_tr_w8_graphs.txt" 2>&1 || { echo "ngd w8 graphs failed"; tail -5 "$OUT/ngd_tr_w8_graphs.txt"; exit 1; }
tail -12 "$OUT/ngd_tr_w8_graphs.txt"
timeout -k 10 300 python scripts/bench_ngd.py --model transformer --world 8 > "$OUT/ngd_tr_w8_eager.txt" 2>&1 || { echo "ngd w8 failed"; tail -5 "$OUT/ngd_tr_w8_eager.txt"; exit 1; }
tail -6 "$OUT/ngd_tr_w8_eager.txt"
timeout -k 10 300 python scripts/bench_ngd.py --model resnet50 --world 8 --graphs > "$OUT/ngd_r50_w8_graphs.txt" 2>&1 || { echo "ngd r50 w8 failed"; tail -5 "$OUT/ngd_r50_w8_graphs.txt"; exit 1; }
tail -6 "$OUT/ngd_r50_w8_graphs.txt"
echo done
