#!/bin/bash
# C4 mix in 1M-frame calls (c4_1m's shape): pipelined async and one-stream, kernel traces
set -u
cd "${GRAFT_REPO_ROOT}"
R=$(pwd); OUT=$R/gpurun_out/r6o; mkdir -p "$OUT"; export TMPDIR=/tmp
cd /tmp
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d "$OUT/async" -o run -- python3 "$R/tools/c4_small_calls.py" --frames 1048576 --calls 100 --warmup 10 > "$OUT/async.log" 2>&1 || exit 1
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d "$OUT/sync" -o run -- python3 "$R/tools/c4_small_calls.py" --frames 1048576 --calls 100 --warmup 10 --sync > "$OUT/sync.log" 2>&1 || exit 1
grep Mpackets "$OUT/async.log" "$OUT/sync.log"
