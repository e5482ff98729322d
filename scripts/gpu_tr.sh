#!/usr/bin/env bash
# Transformer iteration on one GPU: epilogue / attention / graph tests, then the bench
# (graphs on and off).  Usage: bash scripts/gpu_tr.sh [outdir]
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/${1:-tr}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_fused_epilogues.py tests/test_transformer_graphs.py tests/test_attention_gpu.py tests/test_linear.py -x -v -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
timeout -k 10 300 python bench.py --model transformer --steps 20 --warmup 12 > $O/bench_g.log 2>&1 || { tail -30 $O/bench_g.log; exit 1; }
tail -1 $O/bench_g.log
FDT_TR_GRAPHS=0 timeout -k 10 300 python bench.py --model transformer --steps 20 --warmup 12 > $O/bench_nog.log 2>&1 || { tail -30 $O/bench_nog.log; exit 1; }
tail -1 $O/bench_nog.log
