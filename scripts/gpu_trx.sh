#!/usr/bin/env bash
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${1:-trx}
mkdir -p "$OUT"
for i in 1 2 3; do
timeout -k 10 300 python bench.py --model transformer --steps 20 --warmup 12 > "$OUT/bench_tr$i.log" 2>&1 || { tail "$OUT/bench_tr$i.log"; exit 1; }
done
grep -h '"value"' "$OUT"/bench_tr*.log | python3 -c "import sys,json; [print(json.loads(l)['ms_per_step']) for l in sys.stdin]"
