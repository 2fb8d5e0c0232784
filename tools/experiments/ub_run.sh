#!/bin/bash
# GPU box: run the ubench_ws variants given as arguments (default 8_1_4); stop at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
CFG=${CFG:-2}
for v in ${VS:-8_3}; do
  echo "== $v"
  timeout -k 10 120 tools/ubench_ws_$v $CFG 1048576 8 200 > gpurun_out/ub_$v.log 2>&1 || { echo "rc=$?"; tail gpurun_out/ub_$v.log; exit 1; }
  cat gpurun_out/ub_$v.log
done
