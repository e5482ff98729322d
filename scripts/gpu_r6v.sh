#!/usr/bin/env bash
# Round 6: kernel traces of the simulated world-8 ranks (transformer B=32 rank 7, NGD+meta rank 7
# and rank 5) for the per-rank time budget.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r6v}
mkdir -p "$OUT"
timeout -k 10 300 rocprofv3 --kernel-trace -d "$OUT/kt_tr_r7" -o kt -- python bench.py --model transformer --simulate-world 8 --simulate-rank 7 --steps 20 --warmup 15 > "$OUT/kt_tr_r7.log" 2>&1 || { echo "trace tr failed"; tail -5 "$OUT/kt_tr_r7.log"; exit 1; }
python scripts/kstats_db.py "$OUT/kt_tr_r7/kt_results.db" --marker sgd --steps 10 --top 45 > "$OUT/kstats_tr_r7.txt"; head -1 "$OUT/kstats_tr_r7.txt"; rm -rf "$OUT/kt_tr_r7"
for r in 7 5; do
  timeout -k 10 300 rocprofv3 --kernel-trace -d "$OUT/kt_ngd_r$r" -o kt -- python bench.py --ngd --meta_learning --simulate-world 8 --simulate-rank $r --steps 16 --warmup 16 > "$OUT/kt_ngd_r$r.log" 2>&1 || { echo "trace ngd failed"; tail -5 "$OUT/kt_ngd_r$r.log"; exit 1; }
  python scripts/kstats_db.py "$OUT/kt_ngd_r$r/kt_results.db" --marker sgd --steps 8 --top 45 > "$OUT/kstats_ngd_r$r.txt"; head -1 "$OUT/kstats_ngd_r$r.txt"; rm -rf "$OUT/kt_ngd_r$r"
done
echo done
