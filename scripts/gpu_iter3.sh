#!/usr/bin/env bash
# Round-3 iteration: selected GPU tests (-s for printed diagnostics), then the 1-GPU bench at
# bs 1024 / bs 128; optional kernel profile at bs128.
#   bash scripts/gpu_iter3.sh OUT "tests..." [PROF]
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${1:-iter3}; TESTS=${2:-tests/test_conv_kernels.py tests/test_resnet_engine.py}; PROF=${3:-0}
mkdir -p "$OUT"
timeout -k 10 500 python -u -m pytest $TESTS -x -v -s -p no:cacheprovider --timeout 200 --timeout-method thread > "$OUT/pytest.log" 2>&1; rc=$?
grep -E "passed|failed|error|worst" "$OUT/pytest.log" | tail -8
case $rc in 0) ;; 1) echo "tests failed"; grep -E "^(FAILED|E )" "$OUT/pytest.log" | head -20 ;; *) echo "pytest aborted rc=$rc"; tail -20 "$OUT/pytest.log"; exit 1;; esac
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > "$OUT/bench.log" 2>&1 || { tail "$OUT/bench.log"; exit 1; }
timeout -k 10 300 python bench.py --steps 30 --warmup 5 --global-batch 128 > "$OUT/bench128.log" 2>&1 || { tail "$OUT/bench128.log"; exit 1; }
grep -h '"value"' "$OUT/bench.log" "$OUT/bench128.log" | python3 -c "import sys,json; [print(json.loads(l)['config']['global_batch'], json.loads(l)['ms_per_step']) for l in sys.stdin]"
if [ "$PROF" = 1 ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof128" -o run -- python3 bench.py --steps 10 --warmup 3 --global-batch 128 > "$OUT/prof128.log" 2>&1 || { echo prof failed; exit 1; }
  f=$(find "$OUT/prof128" -name '*kernel_stats.csv' | head -n 1); python scripts/kstats.py "$f" --steps 13 --top 60 > "$OUT/kstats128.txt"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- python3 bench.py --steps 4 --warmup 3 > "$OUT/prof.log" 2>&1 || { echo prof failed; exit 1; }
  f=$(find "$OUT/prof" -name '*kernel_stats.csv' | head -n 1); python scripts/kstats.py "$f" --steps 7 --top 60 > "$OUT/kstats1024.txt"
fi
echo done
