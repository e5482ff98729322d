#!/usr/bin/env bash
# CPU sanitizer builds of the host-only runtime code (csrc/runtime/ordered_worker.h: the
# staging worker thread and the DDP bucket planner) -- GPU ASan / XNACK runs are not available
# on this pool, so the host side is checked on its own:
#   1. AddressSanitizer + UndefinedBehaviorSanitizer
#   2. ThreadSanitizer (the worker / submitter hand-off)
# usage: scripts/host_sanitize.sh [OUTDIR]      (exit 0 = clean)
set -euo pipefail
cd "$(dirname "$0")/.."
OUT=${1:-build/sanitize}
mkdir -p "$OUT"
CXX=${CXX:-g++}
"$CXX" -std=c++17 -O1 -g -fno-omit-frame-pointer -fsanitize=address,undefined -fno-sanitize-recover=all \
  -pthread tools/host_selftest.cpp -o "$OUT/host_selftest_asan"
ASAN_OPTIONS=detect_leaks=1:abort_on_error=1 UBSAN_OPTIONS=print_stacktrace=1 "$OUT/host_selftest_asan"
"$CXX" -std=c++17 -O1 -g -fsanitize=thread -pthread tools/host_selftest.cpp -o "$OUT/host_selftest_tsan"
TSAN_OPTIONS=halt_on_error=1 "$OUT/host_selftest_tsan"
echo "host sanitizers: clean"
