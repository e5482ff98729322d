#!/bin/bash
# first GPU validation pass: kernel tests, smoke, bench (native + ablation)
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -m pytest tests/test_gpu_kernels.py -x -q -m gpu > gpurun_out/t1_pytest.log 2>&1
echo "pytest rc=$?" >> gpurun_out/t1_pytest.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/t1_smoke.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/t1_bench.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-native > gpurun_out/t1_bench_nonative.log 2>&1
exit 0
