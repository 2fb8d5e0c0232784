#!/bin/bash
# C4 mix through the pipelined fused call at 1M and 10M frames per call, kernel trace of each
set -u
cd "${GRAFT_REPO_ROOT}"
R=$(pwd); OUT=$R/gpurun_out/profsmall; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 120 python3 tools/c4_small_calls.py --frames 1048576 --calls 200 > "$OUT/plain_1m.json" 2>&1 || exit 1
timeout -k 10 120 python3 tools/c4_small_calls.py --frames 10485760 --calls 20 > "$OUT/plain_10m.json" 2>&1 || exit 1
cat "$OUT/plain_1m.json" "$OUT/plain_10m.json"
cd /tmp
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d "$OUT/t1m" -o run -- python3 "$R/tools/c4_small_calls.py" --frames 1048576 --calls 200 > "$OUT/t1m.log" 2>&1 || exit 1
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d "$OUT/t10m" -o run -- python3 "$R/tools/c4_small_calls.py" --frames 10485760 --calls 20 > "$OUT/t10m.log" 2>&1 || exit 1
find "$OUT" -name "*kernel_stats.csv"
