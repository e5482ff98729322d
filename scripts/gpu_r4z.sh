#!/usr/bin/env bash
# Round 4: multi-rank rehearsal on one GPU (gloo, ranks share cuda:0): the N > 1 code paths of
# bench.py end to end (self-launched torchrun), and sharded NGD with graph replay at world 2.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r4z}
mkdir -p "$OUT"
timeout -k 10 700 python -u -m pytest tests/test_distributed_gpu.py -k "sharded_ngd_graphs_world2" -m gpu -v -p no:cacheprovider \
  --timeout 650 --timeout-method thread > "$OUT/pytest.log" 2>&1; rc=$?
echo "pytest rc=$rc"; tail -1 "$OUT/pytest.log"
case $rc in 0) ;; 1) grep -E "^(FAILED|ERROR)|Error|assert" "$OUT/pytest.log" | head -30; exit 1;; *) echo aborted; tail -20 "$OUT/pytest.log"; exit 1;; esac
run() {
  local name=$1; shift
  FDT_DIST_BACKEND=gloo timeout -k 10 400 python bench.py "$@" > "$OUT/$name.log" 2>&1 || { echo "$name failed"; tail -15 "$OUT/$name.log"; exit 1; }
  grep -h '"value"' "$OUT/$name.log" > "$OUT/$name.json"
  echo "$name $(grep -o '"n_gpus": [0-9]*' "$OUT/$name.json") $(grep -o '"dist_world": [0-9]*' "$OUT/$name.json") $(grep -o '"ms_per_step": [0-9.]*' "$OUT/$name.json")"
}
run dp4 --gpus 4 --steps 3 --warmup 3
run ngd4 --gpus 4 --ngd --meta_learning --steps 4 --warmup 14
run fsdp4 --gpus 4 --fsdp --steps 3 --warmup 3
run tr4 --gpus 4 --model transformer --steps 3 --warmup 6
echo done
