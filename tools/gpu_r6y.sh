#!/bin/bash
# C4 uniform vs Zipf(1.1), table-only, 10.5M-frame calls: one-stream and pipelined kernel traces
set -u
cd "${GRAFT_REPO_ROOT}"
R=$(pwd); OUT=$R/gpurun_out/r6y; mkdir -p "$OUT"; export TMPDIR=/tmp
cd /tmp
for z in u z; do
  ZA=""; [ $z = z ] && ZA="--zipf 1.1"
  for m in sync async; do
    MA=""; [ $m = sync ] && MA="--sync"
    timeout -k 10 180 rocprofv3 --kernel-trace -d "$OUT/${z}_$m" -o run -- python3 "$R/tools/c4_small_calls.py" --frames 10485760 --calls 10 --warmup 2 $ZA $MA > "$OUT/${z}_$m.log" 2>&1 || exit 1
    echo "$z $m $(grep frames_per_call $OUT/${z}_$m.log)"
  done
done
