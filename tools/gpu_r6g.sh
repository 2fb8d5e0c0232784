#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT}"
R=$(pwd); mkdir -p gpurun_out/r6g; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_timed.py tests/test_gpu_c5.py -v --timeout 200 --timeout-method thread > gpurun_out/r6g/tests.txt 2>&1
rc=$?; tail -8 gpurun_out/r6g/tests.txt
if [ $rc -ne 0 ]; then exit $rc; fi
cd /tmp
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/r6g/t10m" -o run -- python3 "$R/tools/c4_small_calls.py" --frames 10485760 --calls 10 --warmup 2 --sync --timed > "$R/gpurun_out/r6g/t10m.log" 2>&1 || exit 1
timeout -k 10 120 python3 "$R/tools/c4_small_calls.py" --frames 10485760 --calls 20 --timed > "$R/gpurun_out/r6g/timed_async.json" 2>&1 || exit 1
cat "$R/gpurun_out/r6g/timed_async.json"
