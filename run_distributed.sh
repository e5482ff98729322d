#!/usr/bin/env bash
# Single-node multi-GPU launch (reference run_distributed.sh:1-3): one rank per MI355X over
# RCCL/xGMI via torchrun.  Reference used 4 GPUs with --bs 256 (global 1024) and
# --batch_size 64 (global 256); with 8 GPUs the same global batches are --bs 128 / -b 32.
#   NGPU=8 bash run_distributed.sh           # both workloads
#   NGPU=8 bash run_distributed.sh resnet    # one of them
#   MAX_RESTARTS=3 bash run_distributed.sh resnet --auto_resume
#       elastic restarts: a failed/killed rank restarts the whole job, which resumes from the
#       full-state checkpoint of the last completed epoch (checkpoint/*_last.pth)
set -euo pipefail
cd "$(dirname "$0")"
NGPU=${NGPU:-$(python -c "import torch; print(max(1, torch.cuda.device_count()))")}
PORT=${MASTER_PORT:-12355}
export HSA_ENABLE_IPC_MODE_LEGACY=0 OMP_NUM_THREADS=${OMP_NUM_THREADS:-12}
RUN="python -m torch.distributed.run --nnodes=1 --nproc_per_node=${NGPU} --master-addr 127.0.0.1 --master_port=${PORT} --max-restarts=${MAX_RESTARTS:-0}"
WHAT=${1:-all}
if [[ "$WHAT" == all || "$WHAT" == resnet ]]; then
  $RUN ./resnet50_test.py --workers 4 --bs $((1024 / NGPU)) --distributed --meta_learning --ngd --lr 0.01 "${@:2}"
fi
if [[ "$WHAT" == all || "$WHAT" == transformer ]]; then
  $RUN ./transformer_test.py --workers 4 --batch_size $((256 / NGPU)) --distributed --ngd "${@:2}"
fi
