#!/usr/bin/env bash
# Round 4: transformer FSDP as ONE unit (the reference's FSDP(model)) vs per-sublayer units.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r4t}
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests/test_distributed_gpu.py -k "transformer_fsdp" -m gpu -v -p no:cacheprovider \
  --timeout 500 --timeout-method thread > "$OUT/pytest.log" 2>&1; rc=$?
echo "pytest rc=$rc"; tail -1 "$OUT/pytest.log"
case $rc in 0) ;; 1) grep -E "^(FAILED|ERROR)|Error" "$OUT/pytest.log" | head -30; exit 1;; *) echo aborted; exit 1;; esac
run() {
  local name=$1; shift
  timeout -k 10 300 python bench.py "$@" > "$OUT/$name.log" 2>&1 || { echo "$name failed"; tail -5 "$OUT/$name.log"; exit 1; }
  grep -h '"value"' "$OUT/$name.log" > "$OUT/$name.json"
  echo "$name $(grep -o '"ms_per_step": [0-9.]*' "$OUT/$name.json") $(grep -o '"host_ms_per_step": [0-9.]*' "$OUT/$name.json")"
}
run tr_fsdp_sublayer --model transformer --fsdp --steps 20 --warmup 12
run tr_fsdp_model --model transformer --fsdp --fsdp-wrap model --steps 20 --warmup 12
run tr_fsdp_model_sgo --model transformer --fsdp --fsdp-wrap model --fsdp-schedule shard_grad_op --steps 20 --warmup 12
echo done
