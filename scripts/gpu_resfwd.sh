#!/usr/bin/env bash
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${1:-resfwd}
mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_resnet_engine.py tests/test_deterministic.py tests/test_conv_kernels.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
for i in 1 2; do
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > "$OUT/bench$i.log" 2>&1 || exit 1
timeout -k 10 300 python bench.py --steps 30 --warmup 5 --global-batch 128 > "$OUT/bench128_$i.log" 2>&1 || exit 1
done
grep -h '"value"' "$OUT"/bench*.log | python3 -c "import sys,json; [print(json.loads(l)['config']['global_batch'], json.loads(l)['ms_per_step']) for l in sys.stdin]"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- python3 bench.py --steps 4 --warmup 3 > "$OUT/prof.log" 2>&1 || exit 1
f=$(find "$OUT/prof" -name '*kernel_stats.csv' | head -n 1); python scripts/kstats.py "$f" --steps 7 --top 40 | grep residual
