#!/usr/bin/env bash
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r5dbg}
mkdir -p "$OUT"
T=tests/test_distributed_gpu.py::test_transformer_ddp_hip_graphs_two_ranks
for cfg in "base:" "noadj:FDT_FLAT_ADJACENT=0" "noprep:FDT_TR_MIXUP_PREP=0" "nometer:FDT_TR_GRAPH_METER=0" "nographs:FDT_TR_GRAPHS=0"; do
  name=${cfg%%:*}; envs=${cfg#*:}
  env $envs timeout -k 10 300 python -u -m pytest $T -q -p no:cacheprovider --timeout 250 --timeout-method thread > "$OUT/$name.log" 2>&1; rc=$?
  echo "$name rc=$rc $(tail -1 $OUT/$name.log)"
  case $rc in 0|1) ;; *) exit 1;; esac
done
