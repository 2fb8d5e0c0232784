#!/bin/bash
# GPU box: the C2 bench line at the driver's settings (--steps 20) under a kernel trace, its warmup
# one launch of the same size (so the parse kernel's average duration is the bench's
# kernel_ms_per_launch of the same command), extras off; the JSON line is kept next to the trace.
set -u
cd "${GRAFT_REPO_ROOT}"
R=$(pwd); OUT=$R/gpurun_out/profdrv; rm -rf "$OUT"; mkdir -p "$OUT"; export TMPDIR=/tmp
cd /tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run -- python3 "$R/bench.py" --steps 20 --warmup 20 \
  --no-cpu-baseline --no-imix --no-other-mode --no-host --no-single-launch > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail "$OUT/bench.err"; exit 1; }
tail -c 400 "$OUT/bench.json"
