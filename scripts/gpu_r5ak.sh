#!/usr/bin/env bash
# Fused update-and-pack as two launches (1x1 at a 4 KB LDS image, 3x3 at 38 KB): tests + A/B.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r5ak}
mkdir -p "$OUT"
FDT_NATIVE=1 timeout -k 10 120 python -c "from faster_distributed_training_amd.ops import _native; _native.native()" || { echo "native extension stale or missing"; exit 1; }
timeout -k 10 600 python -u -m pytest tests/test_optim_pack.py tests/test_optim.py tests/test_conv_kernels.py -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1; rc=$?
echo "pytest rc=$rc"; tail -1 "$OUT/pytest.log"; grep -E "^(FAILED|ERROR)" "$OUT/pytest.log" | head
[ $rc -eq 0 ] || exit 1
run() {
  local name=$1; shift
  timeout -k 10 300 python bench.py "$@" > "$OUT/$name.log" 2>&1 || { echo "$name failed"; tail -5 "$OUT/$name.log"; exit 1; }
  grep -h '"value"' "$OUT/$name.log" > "$OUT/$name.json"
  echo "$name $(grep -o '"ms_per_step": [0-9.]*' "$OUT/$name.json")"
}
FDT_PACK_IN_OPT=0 run bs128_off_a --steps 40 --warmup 5 --global-batch 128
FDT_PACK_IN_OPT=1 run bs128_on_a --steps 40 --warmup 5 --global-batch 128
FDT_PACK_IN_OPT=0 run bs128_off_b --steps 40 --warmup 5 --global-batch 128
FDT_PACK_IN_OPT=1 run bs128_on_b --steps 40 --warmup 5 --global-batch 128
FDT_PACK_IN_OPT=0 run bs1024_off --steps 30 --warmup 8
FDT_PACK_IN_OPT=1 run bs1024_on --steps 30 --warmup 8
FDT_PACK_IN_OPT=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_bs128" -o run -- python3 bench.py --steps 10 --warmup 5 --global-batch 128 > "$OUT/prof_bs128.log" 2>&1 || { echo "prof failed"; tail -5 "$OUT/prof_bs128.log"; exit 1; }
f=$(find "$OUT/prof_bs128" -name '*kernel_stats.csv' | head -n 1)
python scripts/kstats.py "$f" --steps 15 --top 80 > "$OUT/kstats_bs128.txt"
grep -E "pack|madgrad" "$OUT/kstats_bs128.txt" | cut -c1-150
echo done
