#!/usr/bin/env bash
# Quick GPU iteration: selected tests, then the 1-GPU bench at bs 1024 and bs 128 (+ optional profile).
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${1:-quick}; TESTS=${2:-tests/test_conv_kernels.py tests/test_resnet_engine.py}; PROF=${3:-0}
mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest $TESTS -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > "$OUT/bench.log" 2>&1 || { tail "$OUT/bench.log"; exit 1; }
timeout -k 10 300 python bench.py --steps 30 --warmup 5 --global-batch 128 > "$OUT/bench128.log" 2>&1 || { tail "$OUT/bench128.log"; exit 1; }
grep -h '"value"' "$OUT/bench.log" "$OUT/bench128.log" | python3 -c "import sys,json; [print(json.loads(l)['config']['global_batch'], json.loads(l)['ms_per_step']) for l in sys.stdin]"
if [ "$PROF" = 1 ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- python bench.py --steps 4 --warmup 3 > "$OUT/prof.log" 2>&1 || { echo prof failed; exit 1; }
fi
echo done
