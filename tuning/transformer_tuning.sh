#!/usr/bin/env bash
# lr x weight-decay grid on a 10% subset, 5 epochs, NGD (reference
# tuning/transformer_tuning.sh; its echo line misspelled --weighted_decay).
set -euo pipefail
cd "$(dirname "$0")"
for lr in 1e-4 1e-3 1e-2; do
  for wd in 5e-4 1e-4 5e-3; do
    echo "lr=${lr} weight_decay=${wd}"
    python ./transformer_tuning.py --workers 4 --batch_size 64 --ngd --lr "$lr" --weight_decay "$wd" --epoch 5 "$@"
  done
done
