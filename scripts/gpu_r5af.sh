#!/usr/bin/env bash
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r5af}
mkdir -p "$OUT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_tr_b256" -o run -- python3 bench.py --model transformer --steps 8 --warmup 12 > "$OUT/prof_tr_b256.log" 2>&1 || { echo "prof failed"; tail -5 "$OUT/prof_tr_b256.log"; exit 1; }
f=$(find "$OUT/prof_tr_b256" -name '*kernel_stats.csv' | head -n 1)
python scripts/kstats.py "$f" --steps 20 --top 45 > "$OUT/kstats_tr_b256.txt"
head -45 "$OUT/kstats_tr_b256.txt" | cut -c1-150
FDT_NATIVE=1 timeout -k 10 120 python -c "from faster_distributed_training_amd.ops import _native; _native.native()" || { echo "native extension stale or missing"; exit 1; }
for b in 128 1024; do
timeout -k 10 300 python -u scripts/ring_probe.py --batch $b > "$OUT/ring_probe_bs$b.txt" 2>&1 || { echo "ring probe failed"; tail -5 "$OUT/ring_probe_bs$b.txt"; exit 1; }
cat "$OUT/ring_probe_bs$b.txt" | cut -c1-400
done
echo done
