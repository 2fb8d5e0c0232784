#!/bin/bash
# C5 merge timing + GPU C5 test, then the history kernel variants.
set -u
cd "${GRAFT_REPO_ROOT}"; R=$(pwd); export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_c5.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/c5_test.log 2>&1 || { tail -20 gpurun_out/c5_test.log; exit 1; }
tail -2 gpurun_out/c5_test.log
timeout -k 10 300 python -u tools/c5_merge_time.py > gpurun_out/c5_merge_time.log 2>&1 || { tail -20 gpurun_out/c5_merge_time.log; exit 1; }
grep merge gpurun_out/c5_merge_time.log
VARS="${VARS:-product nobatch norank}" bash tools/experiments/r3_histvar.sh
