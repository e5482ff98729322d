#!/usr/bin/env bash
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${1:-detbench}
mkdir -p "$OUT"
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --deterministic > "$OUT/det1024.log" 2>&1 || exit 1
timeout -k 10 300 python bench.py --steps 30 --warmup 5 --global-batch 128 --deterministic > "$OUT/det128.log" 2>&1 || exit 1
grep -h '"value"' "$OUT"/det*.log | python3 -c "import sys,json; [print(json.loads(l)['config']['global_batch'], json.loads(l)['ms_per_step'], json.loads(l)['config'].get('deterministic')) for l in sys.stdin]"
