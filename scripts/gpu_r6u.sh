#!/usr/bin/env bash
# Round 6: counters of the slow stage-3/4 1x1 layers at batch 1024.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
bash scripts/pmc_layer.sh r6u/fwd_8x8_256_1024 fwd 8,256,1024,1,1,0 || exit 1
bash scripts/pmc_layer.sh r6u/wgrad_8x8_1024_256 wgrad 8,1024,256,1,1,0 || exit 1
bash scripts/pmc_layer.sh r6u/fwd_4x4_512_2048 fwd 4,512,2048,1,1,0 || exit 1
