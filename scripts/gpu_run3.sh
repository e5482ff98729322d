#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -m pytest tests/test_gpu_kernels.py -q -m gpu -k "stats or act_bwd or residual or fp32_matches" > gpurun_out/t3_pytest.log 2>&1
echo "pytest rc=$?" >> gpurun_out/t3_pytest.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/t3_bench.log 2>&1 || exit 1
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof3 -o run --output-format csv -- python bench.py --steps 4 --warmup 3 > gpurun_out/t3_prof.log 2>&1
exit 0
