#!/usr/bin/env bash
# Hyper-parameter grid on a 10% strided CIFAR subset, 5 epochs, NGD (reference
# tuning/resnet50_tuning.sh: alpha x gamma grid with StepLR(2, gamma)).
set -euo pipefail
cd "$(dirname "$0")"
for alpha in 0.99 0.9 0.8; do
  for gamma in 0.75 0.85 0.95; do
    echo "alpha=${alpha} gamma=${gamma}"
    python ./resnet50_tuning.py --workers 4 --bs 256 --ngd --alpha "$alpha" --gamma "$gamma" --epoch 5 "$@"
  done
done
