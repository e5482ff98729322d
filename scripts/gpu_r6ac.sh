#!/usr/bin/env bash
# Round 6: halo weight gradient, tap split over two waves (TS = 2) x fragment pipeline.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r6ac}
mkdir -p "$OUT"
FDT_NATIVE=1 timeout -k 10 120 python -c "from faster_distributed_training_amd.ops import _native; _native.native()" || { echo "native extension stale or missing"; exit 1; }
FDT_WGRAD_H3_TS=2 timeout -k 10 300 python -u -m pytest tests/test_conv_kernels.py -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "h3_conv_wgrad" > "$OUT/pytest_wh3_ts2.log" 2>&1; rc=$?
echo "pytest wh3 ts2 rc=$rc"; tail -1 "$OUT/pytest_wh3_ts2.log"
case $rc in 0|1) grep -E "^FAILED" "$OUT/pytest_wh3_ts2.log" | head -20;; *) echo aborted; tail -20 "$OUT/pytest_wh3_ts2.log"; exit 1;; esac
for ts in 1 2; do
  for pp in 0 1; do
    for b in 1024 128; do
      FDT_WGRAD_H3_TS=$ts FDT_WGRAD_H3_PIPE=$pp timeout -k 10 300 python -u scripts/bench_h3.py --batch $b --only wgrad > "$OUT/wh3_ts${ts}_p${pp}_$b.txt" 2>&1 || { echo "bench failed"; tail -5 "$OUT/wh3_ts${ts}_p${pp}_$b.txt"; exit 1; }
      echo "ts $ts pipe $pp batch $b: $(grep -o 'halo ((.*' $OUT/wh3_ts${ts}_p${pp}_$b.txt | sed 's/halo ((\([0-9]*\), \([0-9]*\)), [0-9]*): *\([0-9.]*\) us ( *[0-9]* TF\/s, \(.*\))/\1x\2 \3us d=\4/' | tr '\n' ' ')"
    done
  done
done
