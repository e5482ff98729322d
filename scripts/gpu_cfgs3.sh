#!/usr/bin/env bash
# Round-3 config benches: FSDP (world-1 group, sharded path active), sharded NGD at world 1,
# NGD+meta dp1, transformer B=256 and B=32.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${1:-cfgs3}; shift
mkdir -p "$OUT"
run() { local name=$1; shift; timeout -k 10 300 python bench.py "$@" > "$OUT/$name.log" 2>&1 || { echo "$name failed"; tail -5 "$OUT/$name.log"; return 1; }; grep -h '"value"' "$OUT/$name.log" | python3 -c "import sys,json; r=json.loads(sys.stdin.read()); print('$name', r['ms_per_step'], 'ms', {k: v for k, v in r['config'].items() if k.startswith(('fsdp', 'owner', 'ddp', 'optimizer_sh', 'ngd_'))})"; }
for c in "$@"; do
  case $c in
    fsdp) run fsdp --fsdp --steps 20 --warmup 5 ;;
    fsdp128) run fsdp128 --fsdp --steps 30 --warmup 5 --global-batch 128 ;;
    ngd) run ngd --ngd --meta_learning --steps 20 --warmup 15 ;;
    zero) run zero --ngd --meta_learning --sharded-ngd --steps 20 --warmup 15 ;;
    tr) run tr --model transformer --steps 20 --warmup 12 ;;
    tr32) run tr32 --model transformer --global-batch 32 --steps 40 --warmup 12 ;;
    tr_nog) FDT_NGD_GRAPHS=0 run tr_nog --model transformer --steps 20 --warmup 12 ;;
    tr32_nog) FDT_NGD_GRAPHS=0 run tr32_nog --model transformer --global-batch 32 --steps 40 --warmup 12 ;;
    dp) run dp --steps 20 --warmup 5 ;;
    dp128) run dp128 --steps 30 --warmup 5 --global-batch 128 ;;
  esac || exit 1
done
echo done
