#!/usr/bin/env bash
# A/B of an engine env switch on the 1-GPU bench (interleaved runs, same box).
# usage: scripts/ab_bench.sh OUTDIR VAR VALUE_A VALUE_B [bench args...]
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/$1; VAR=$2; A=$3; B=$4; shift 4
mkdir -p "$OUT"
for r in 1 2; do
  for v in "$A" "$B"; do
    env "$VAR=$v" timeout -k 10 300 python bench.py "$@" > "$OUT/${VAR}_${v}_$r.log" 2>&1 || { echo "bench $v failed"; exit 1; }
  done
done
grep -h '"value"' "$OUT"/*.log | python3 -c "import sys,json; [print(json.loads(l)['ms_per_step']) for l in sys.stdin]"
ls "$OUT"
