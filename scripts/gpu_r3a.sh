#!/usr/bin/env bash
# Round-3 baseline: bs1024 / bs128 benches and a bs128 kernel profile.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r3a}
mkdir -p "$OUT"
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > "$OUT/bench.log" 2>&1 || { tail "$OUT/bench.log"; exit 1; }
timeout -k 10 300 python bench.py --steps 30 --warmup 5 --global-batch 128 > "$OUT/bench128.log" 2>&1 || { tail "$OUT/bench128.log"; exit 1; }
grep -h '"value"' "$OUT/bench.log" "$OUT/bench128.log" | cut -c1-200
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof128" -o run -- python3 bench.py --steps 10 --warmup 3 --global-batch 128 > "$OUT/prof128.log" 2>&1 || { echo prof failed; exit 1; }
f=$(find "$OUT/prof128" -name '*kernel_stats.csv' | head -n 1); python scripts/kstats.py "$f" --steps 13 --top 60 > "$OUT/kstats128.txt"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- python3 bench.py --steps 4 --warmup 3 > "$OUT/prof.log" 2>&1 || { echo prof failed; exit 1; }
f=$(find "$OUT/prof" -name '*kernel_stats.csv' | head -n 1); python scripts/kstats.py "$f" --steps 7 --top 60 > "$OUT/kstats1024.txt"

timeout -k 10 400 python -u -m pytest tests/test_distributed_gpu.py tests/test_provenance.py -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > "$OUT/pytest_dist.log" 2>&1; echo "pytest rc=$?"; tail -5 "$OUT/pytest_dist.log"
echo done
