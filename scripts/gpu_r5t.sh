#!/usr/bin/env bash
# Jacobi sweeps on the real NGD matrices + a fresh bs128 kernel profile.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r5t}
mkdir -p "$OUT"
FDT_NATIVE=1 timeout -k 10 120 python -c "from faster_distributed_training_amd.ops import _native; _native.native()" || { echo "native extension stale or missing"; exit 1; }
for m in transformer resnet50; do
timeout -k 10 300 python -u scripts/eigh_probe.py --model $m > "$OUT/eigh_probe_$m.txt" 2>&1 || { echo "eigh probe $m failed"; tail -5 "$OUT/eigh_probe_$m.txt"; exit 1; }
cat "$OUT/eigh_probe_$m.txt"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_bs128" -o run -- python3 bench.py --steps 10 --warmup 5 --global-batch 128 > "$OUT/prof_bs128.log" 2>&1 || { echo "prof failed"; tail -5 "$OUT/prof_bs128.log"; exit 1; }
f=$(find "$OUT/prof_bs128" -name '*kernel_stats.csv' | head -n 1)
python scripts/kstats.py "$f" --steps 15 --top 70 > "$OUT/kstats_bs128.txt"
head -3 "$OUT/kstats_bs128.txt"
echo done
