#!/usr/bin/env bash
# Round 4, second call: the new GPU tests (DDP collectives captured in the backward graph, FSDP full-shard ring under
# graphs, transformer under static FSDP, batch-128 shipped tile table, fp16 CE), convergence
# parity, DDP capture-vs-cut at batch 128, FSDP schedules, transformer FSDP, NGD shard graphs.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r4b}
mkdir -p "$OUT"
timeout -k 10 900 python -u -m pytest tests/test_distributed_gpu.py tests/test_resnet_engine.py tests/test_transformer_graphs.py \
  tests/test_gpu_kernels.py::test_ngd_gram_and_wupdate_match_fp64 tests/test_ngd_graphs.py tests/test_conv_kernels.py::test_conv_wgrad -m gpu -v -p no:cacheprovider --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 "$OUT/pytest.log"
case $rc in 0|1) ;; *) echo "pytest aborted rc=$rc"; exit 1;; esac
grep -E "^(FAILED|ERROR)" "$OUT/pytest.log" | head -20
run() {
  local name=$1; shift
  timeout -k 10 300 python bench.py "$@" > "$OUT/$name.log" 2>&1 || { echo "$name failed"; tail -5 "$OUT/$name.log"; exit 1; }
  grep -h '"value"' "$OUT/$name.log" > "$OUT/$name.json"
  echo "$name $(grep -o '"ms_per_step": [0-9.]*' "$OUT/$name.json") $(grep -o '"host_ms_per_step": [0-9.]*' "$OUT/$name.json") $(grep -o '"bwd_graph_segments": [0-9]*' "$OUT/$name.json")"
}
run bs128 --steps 40 --warmup 5 --global-batch 128
FDT_GRAPH_COMM=capture run bs128_ddp_capture --steps 40 --warmup 5 --global-batch 128 --ddp
FDT_GRAPH_COMM=capture run bs1024_ddp_capture --steps 20 --warmup 5 --ddp
FDT_GRAPH_COMM=cut run bs128_ddp_cut --steps 40 --warmup 5 --global-batch 128 --ddp
run fsdp_full --fsdp --steps 10 --warmup 3
run fsdp_sgo --fsdp --fsdp-schedule shard_grad_op --steps 10 --warmup 3
run tr_fsdp --model transformer --fsdp --steps 20 --warmup 12
run tr_b256 --model transformer --steps 20 --warmup 12
run tr_b32 --model transformer --global-batch 32 --steps 40 --warmup 12
timeout -k 10 400 python -u scripts/convergence.py --steps 300 --out "$OUT/convergence.json" > "$OUT/convergence.log" 2>&1 || { echo convergence failed; tail -5 "$OUT/convergence.log"; exit 1; }
cat "$OUT/convergence.log" | tail -2
timeout -k 10 300 python scripts/bench_ngd.py --world 8 > "$OUT/ngd_w8.txt" 2>&1 && tail -1 "$OUT/ngd_w8.txt"
timeout -k 10 300 python scripts/bench_ngd.py --world 8 --graphs > "$OUT/ngd_w8_graphs.txt" 2>&1 && tail -1 "$OUT/ngd_w8_graphs.txt"
echo done
