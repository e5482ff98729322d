#!/usr/bin/env bash
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${1:-occ}
mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest tests/test_conv_kernels.py tests/test_resnet_engine.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
for i in 1 2; do
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > "$OUT/bench$i.log" 2>&1 || { tail "$OUT/bench$i.log"; exit 1; }
timeout -k 10 300 python bench.py --steps 30 --warmup 5 --global-batch 128 > "$OUT/bench128_$i.log" 2>&1 || { tail "$OUT/bench128_$i.log"; exit 1; }
done
grep -h '"value"' "$OUT"/bench*.log | python3 -c "import sys,json; [print(json.loads(l)['config']['global_batch'], json.loads(l)['ms_per_step']) for l in sys.stdin]"
