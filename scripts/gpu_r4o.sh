#!/usr/bin/env bash
# Round 4: per-layer rooflines of exactly the conv calls one engine step makes (keyed by the
# tuned-table variant, counts from scripts/engine_launch_keys.py).
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r4o}
mkdir -p "$OUT/pmc"
for b in 1024 128; do
  timeout -k 10 300 python scripts/roofline_layers.py --batch $b --keys scripts/engine_keys/keys$b.txt --md "$OUT/pmc/r4_bs${b}_roofline.md" --json "$OUT/pmc/roof$b.json" > "$OUT/roof$b.log" 2>&1 && tail -1 "$OUT/roof$b.log" || { tail -5 "$OUT/roof$b.log"; exit 1; }
done
echo done
