#!/bin/bash
# Round 5: where the one-batch-per-call rate goes -- the C2 line with one batch per launch
# (--batches-per-launch 1) under a kernel trace: per-dispatch durations and the gaps between them.
set -u
cd "${GRAFT_REPO_ROOT}"
R=$(pwd); OUT=$R/gpurun_out/r5single; rm -rf "$OUT"; mkdir -p "$OUT"; export TMPDIR=/tmp
cd /tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run -- python3 "$R/bench.py" --steps 64 --warmup 16 \
  --batches-per-launch 1 --no-cpu-baseline --no-imix --no-other-mode --no-host --no-single-launch --no-c4 --no-copy-ref \
  > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail "$OUT/bench.err"; exit 1; }
tail -c 300 "$OUT/bench.json"
find "$OUT/trace" -name "*kernel_trace.csv" | head -1 | xargs -I{} cp {} "$OUT/kernel_trace.csv"
