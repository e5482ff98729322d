#!/usr/bin/env bash
# RCCL stream priority set in-process (parallel/dist._comm_env): queue ids in a trace of the DDP
# path at world 1, plus the distributed GPU tests.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${1:-ddpq2}
mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest tests/test_distributed_gpu.py -m gpu -q -p no:cacheprovider --timeout 200 --timeout-method thread > "$OUT/pytest.log" 2>&1; rc=$?
tail -1 "$OUT/pytest.log"
case $rc in 0|1) ;; *) echo "pytest aborted rc=$rc"; exit 1;; esac
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/prof" -o run -- python3 bench.py --steps 4 --warmup 3 --global-batch 128 --ddp --bucket-mb 8 > "$OUT/prof.log" 2>&1 || { echo prof failed; tail "$OUT/prof.log"; exit 1; }
f=$(find "$OUT/prof" -name '*kernel_trace.csv' | head -n 1)
python - "$f" <<'PY'
import csv, sys
q = {}
with open(sys.argv[1]) as fh:
    for r in csv.DictReader(fh):
        k = ('rccl' if 'oneRank' in r['Kernel_Name'] else 'other', r['Queue_Id'], r['Stream_Id'])
        q[k] = q.get(k, 0) + 1
print("kernel queue/stream use:", q)
PY
timeout -k 10 300 python bench.py --steps 40 --warmup 5 --global-batch 128 --ddp > "$OUT/b128_ddp25.log" 2>&1 && grep -o '"ms_per_step": [0-9.]*' "$OUT/b128_ddp25.log"
