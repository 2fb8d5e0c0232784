#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT}"
R=$(pwd); OUT=$R/gpurun_out/proftimed; mkdir -p "$OUT"; export TMPDIR=/tmp
cd /tmp
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d "$OUT/t10m" -o run -- python3 "$R/tools/c4_small_calls.py" --frames 10485760 --calls 10 --warmup 2 --sync --timed > "$OUT/t10m.log" 2>&1 || exit 1
grep frames_per_call "$OUT/t10m.log"
