#!/bin/bash
# Round 5: kernel trace of the pipelined C4 line (config 4 main line) with grouped units on / off.
set -u
cd "${GRAFT_REPO_ROOT}"
R=$(pwd); OUT=$R/gpurun_out/r5grpprof; rm -rf "$OUT"; mkdir -p "$OUT"; export TMPDIR=/tmp
cd /tmp
for g in 1 0; do
  FB_UNIT_GROUP=$g timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/g$g" -o run -- python3 "$R/bench.py" --config 4 --steps 10 --warmup 2 --no-cpu-baseline --no-other-mode --no-host --no-imix > "$OUT/g$g.log" 2>&1 || { tail -5 "$OUT/g$g.log"; exit 1; }
  echo "== group=$g"; python3 "$R/tools/rocpd_summary.py" "$OUT/g$g/run_results.db" k_flow_apply | head -12
done
