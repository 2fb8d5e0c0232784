#!/bin/bash
# Round 4: C4 pipelined (fb_process_seg_async_dev) table-only lines, uniform and Zipf(1.1), each
# under a kernel trace.
set -u
cd "${GRAFT_REPO_ROOT}"
R=$(pwd); OUT=$R/gpurun_out/r4c4; rm -rf "$OUT"; mkdir -p "$OUT"; export TMPDIR=/tmp
X="--no-cpu-baseline --no-host --no-imix --no-other-mode --no-single-launch --table-only"
cd /tmp
for v in unif zipf; do
  Z=""; [ $v = zipf ] && Z="--zipf 1.1"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/$v" -o run -- python3 "$R/bench.py" --config 4 $Z --steps 20 --warmup 3 $X > "$OUT/$v.json" 2> "$OUT/$v.err" || { echo "$v failed"; tail -5 "$OUT/$v.err"; exit 1; }
  echo "== $v done"
done
