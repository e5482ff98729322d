#!/usr/bin/env bash
# Round 6: halo weight-gradient split count vs pixels per workgroup (slab size), batch 128 / 1024.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r6aa}
mkdir -p "$OUT"
for c in 1 4 8 16; do
  for b in 128 1024; do
    FDT_WGRAD_H3_MIN_CPS=$c timeout -k 10 300 python -u scripts/bench_h3.py --batch $b --only wgrad > "$OUT/wh3_cps${c}_$b.txt" 2>&1 || { echo "bench failed"; tail -5 "$OUT/wh3_cps${c}_$b.txt"; exit 1; }
    echo "min_cps $c batch $b: $(grep -o 'halo ((.*TF/s' $OUT/wh3_cps${c}_$b.txt | sed 's/ TF\/s//; s/halo //' | tr '\n' ' ')"
  done
done
