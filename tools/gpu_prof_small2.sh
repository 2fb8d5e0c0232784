#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT}"
R=$(pwd); OUT=$R/gpurun_out/profsmall2; mkdir -p "$OUT"; export TMPDIR=/tmp
cd /tmp
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d "$OUT/s1m" -o run -- python3 "$R/tools/c4_small_calls.py" --frames 1048576 --calls 200 --sync > "$OUT/s1m.log" 2>&1 || exit 1
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d "$OUT/s10m" -o run -- python3 "$R/tools/c4_small_calls.py" --frames 10485760 --calls 20 --sync > "$OUT/s10m.log" 2>&1 || exit 1
cat "$OUT/s1m.log" "$OUT/s10m.log" | grep frames_per_call
