#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -m pytest tests/test_gpu_kernels.py -q -m gpu -k "engine" > gpurun_out/t2_pytest.log 2>&1
echo "pytest rc=$?" >> gpurun_out/t2_pytest.log
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof2 -o run --output-format csv -- python bench.py --steps 4 --warmup 3 > gpurun_out/t2_prof.log 2>&1
echo "prof rc=$?" >> gpurun_out/t2_prof.log
exit 0
