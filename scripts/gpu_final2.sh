#!/usr/bin/env bash
# End-of-session evidence: all GPU tests, smoke, benches, kernel profiles, PMC rooflines.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${1:-final2}
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1; rc=$?; echo "pytest rc=$rc" >> "$OUT/pytest.log"; tail -3 "$OUT/pytest.log"
case $rc in 0|1) ;; *) echo "pytest aborted rc=$rc"; exit 1;; esac
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { echo smoke failed; exit 1; }
tail -1 "$OUT/smoke.log"
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > "$OUT/bench.log" 2>&1 || { echo bench failed; exit 1; }
timeout -k 10 300 python bench.py --steps 30 --warmup 5 --global-batch 128 > "$OUT/bench128.log" 2>&1 || { echo bench128 failed; exit 1; }
timeout -k 10 300 python bench.py --model transformer --steps 20 --warmup 12 > "$OUT/bench_tr.log" 2>&1 || { echo bench_tr failed; exit 1; }
timeout -k 10 300 python bench.py --ngd --meta_learning --steps 20 --warmup 15 > "$OUT/bench_ngd_meta.log" 2>&1 || { echo bench_ngd_meta failed; exit 1; }
grep -h '"value"' "$OUT"/bench*.log | cut -c1-150
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- python3 bench.py --steps 4 --warmup 3 > "$OUT/prof.log" 2>&1 || { echo prof failed; exit 1; }
f=$(find "$OUT/prof" -name '*kernel_stats.csv' | head -n 1); python scripts/kstats.py "$f" --steps 7 --top 40 > "$OUT/kstats_resnet.txt"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/proft" -o run -- python3 bench.py --model transformer --steps 10 --warmup 6 > "$OUT/proft.log" 2>&1 || { echo proft failed; exit 1; }
f=$(find "$OUT/proft" -name '*kernel_stats.csv' | head -n 1); python scripts/kstats.py "$f" --steps 16 --top 40 > "$OUT/kstats_tr.txt"
bash scripts/pmc_step.sh final 1024 > "$OUT/pmc1024.log" 2>&1 || { echo pmc1024 failed; tail "$OUT/pmc1024.log"; exit 1; }
bash scripts/pmc_step.sh final 128 > "$OUT/pmc128.log" 2>&1 || { echo pmc128 failed; tail "$OUT/pmc128.log"; exit 1; }
echo done
