#!/usr/bin/env bash
# Round 6: counters of the largest lost-time 1x1 row at batch 1024 (32x32 64->256 forward) and
# of a join-backward vs activation-backward fold-prologue data gradient (bank conflicts).
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
bash scripts/pmc_layer.sh r6aj/fwd_32x32_64_256 fwd 32,64,256,1,1,0 || exit 1
bash scripts/pmc_layer.sh r6aj/dgrad_16x16_128_512 dgrad 16,128,512,1,1,0 || exit 1
