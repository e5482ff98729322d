#!/usr/bin/env bash
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r2s}
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "eigh or ngd" > "$OUT/pytest.log" 2>&1; tail -15 "$OUT/pytest.log"
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- python3 scripts/bench_ngd.py --model resnet50 --steps 40 > "$OUT/prof.log" 2>&1 || { echo prof failed; exit 1; }
f=$(find "$OUT/prof" -name '*kernel_stats.csv' | head -n 1)
python scripts/kstats.py "$f" --steps 40 --top 25 > "$OUT/kstats.txt"; cat "$OUT/kstats.txt"
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/proft" -o run -- python3 scripts/bench_ngd.py --model transformer --steps 40 > "$OUT/proft.log" 2>&1 || { echo prof failed; exit 1; }
f=$(find "$OUT/proft" -name '*kernel_stats.csv' | head -n 1)
python scripts/kstats.py "$f" --steps 40 --top 25 > "$OUT/kstats_tr.txt"; cat "$OUT/kstats_tr.txt"
