#!/usr/bin/env bash
# Round-3 counter tables: ResNet-50 bs1024 and bs128 training steps, calibrated normalisation.
set -o pipefail
cd "$(dirname "$0")/.."
bash scripts/pmc_step.sh r3 1024 > gpurun_out/pmc_r3_1024.log 2>&1 || { echo pmc1024 failed; tail -5 gpurun_out/pmc_r3_1024.log; exit 1; }
bash scripts/pmc_step.sh r3 128 > gpurun_out/pmc_r3_128.log 2>&1 || { echo pmc128 failed; tail -5 gpurun_out/pmc_r3_128.log; exit 1; }
echo done
