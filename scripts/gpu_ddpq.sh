#!/usr/bin/env bash
# Does RCCL's stream share a hardware queue with the compute stream?  DDP at world 1, batch 128,
# default vs high-priority RCCL streams (TORCH_NCCL_HIGH_PRIORITY=1): bench + queue ids in a trace.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${1:-ddpq}
mkdir -p "$OUT"
run() {
  local name=$1 hp=$2; shift 2
  TORCH_NCCL_HIGH_PRIORITY=$hp timeout -k 10 300 python bench.py "$@" > "$OUT/$name.log" 2>&1 || { echo "$name failed"; tail -5 "$OUT/$name.log"; exit 1; }
  grep -h '"value"' "$OUT/$name.log" > "$OUT/$name.json"
  echo "$name $(grep -o '"ms_per_step": [0-9.]*' "$OUT/$name.json") $(grep -o '"ddp_buckets": [0-9]*' "$OUT/$name.json")"
}
run b128_ddp_hp0 0 --steps 40 --warmup 5 --global-batch 128 --ddp --bucket-mb 8
run b128_ddp_hp1 1 --steps 40 --warmup 5 --global-batch 128 --ddp --bucket-mb 8
run b128_ddp25_hp1 1 --steps 40 --warmup 5 --global-batch 128 --ddp
export TORCH_NCCL_HIGH_PRIORITY=1
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/prof" -o run -- python3 bench.py --steps 4 --warmup 3 --global-batch 128 --ddp --bucket-mb 8 > "$OUT/prof.log" 2>&1 || { echo prof failed; tail "$OUT/prof.log"; exit 1; }
f=$(find "$OUT/prof" -name '*kernel_trace.csv' | head -n 1)
python - "$f" <<'PY'
import csv, sys
rows = []
with open(sys.argv[1]) as fh:
    for r in csv.DictReader(fh):
        rows.append((int(r['Start_Timestamp']), int(r['End_Timestamp']), r['Kernel_Name'][:40], r['Queue_Id'], r['Stream_Id']))
rows.sort()
q = {}
for r in rows:
    k = ('rccl' if 'oneRank' in r[2] else 'other', r[3], r[4])
    q[k] = q.get(k, 0) + 1
print("kernel queue/stream use:", q)
ov = sum(1 for a, b in zip(rows, rows[1:]) if b[0] < a[1])
print("overlapping consecutive pairs:", ov, "of", len(rows))
PY
