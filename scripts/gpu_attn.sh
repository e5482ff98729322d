#!/usr/bin/env bash
# Attention kernels: GPU tests, transformer bench and its kernel profile.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${1:-attn}
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest tests/test_attention_gpu.py tests/test_fused_epilogues.py tests/test_transformer_graphs.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
timeout -k 10 300 python bench.py --model transformer --steps 20 --warmup 12 > "$OUT/bench_tr.log" 2>&1 || { tail "$OUT/bench_tr.log"; exit 1; }
grep '"value"' "$OUT/bench_tr.log" | cut -c1-220
bash scripts/prof_tr.sh "$(basename $OUT)_prof" | head -12
