#!/usr/bin/env bash
# NGD fused projection + attention drop bit mask: kernel tests, NGD step bench, transformer bench/profile.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r2q}
mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_attention_gpu.py tests/test_transformer_graphs.py tests/test_fused_epilogues.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { tail -40 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
timeout -k 10 200 python scripts/bench_ngd.py --model resnet50 --steps 40 > "$OUT/bench_ngd.log" 2>&1 || { tail "$OUT/bench_ngd.log"; exit 1; }
timeout -k 10 200 python scripts/bench_ngd.py --model transformer --steps 40 >> "$OUT/bench_ngd.log" 2>&1 || { tail "$OUT/bench_ngd.log"; exit 1; }
grep steps "$OUT/bench_ngd.log"
timeout -k 10 300 python bench.py --model transformer --steps 20 --warmup 12 > "$OUT/bench_tr.log" 2>&1 || { tail "$OUT/bench_tr.log"; exit 1; }
grep '"value"' "$OUT/bench_tr.log" | cut -c1-220
bash scripts/prof_tr.sh "$(basename $OUT)_prof" | head -14
