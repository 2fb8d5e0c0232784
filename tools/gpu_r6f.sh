#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/r6f
timeout -k 10 300 python -u -m pytest tests/test_gpu_queue.py -v --timeout 200 --timeout-method thread > gpurun_out/r6f/queue_tests.txt 2>&1
rc=$?; tail -15 gpurun_out/r6f/queue_tests.txt
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
bash tools/gpu_r6e.sh
