#!/bin/bash
# Round 3 first GPU call: the whole GPU suite, then the K2 cost split (tools/experiments/r3_k2probe.sh).
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r3_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r3_tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/experiments/r3_k2probe.sh
