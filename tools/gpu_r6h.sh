#!/bin/bash
# timed pass at HEAD: timed + C5 GPU tests, then a kernel trace of the timed C4 shape
set -u
cd "${GRAFT_REPO_ROOT}"
R=$(pwd); OUT=$R/gpurun_out/r6h; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_timed.py tests/test_gpu_c5.py -x -v --timeout 120 --timeout-method thread -m gpu > "$OUT/tests.log" 2>&1 || { tail -30 "$OUT/tests.log"; exit 1; }
tail -3 "$OUT/tests.log"
cd /tmp
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d "$OUT/cur" -o run -- python3 "$R/tools/c4_small_calls.py" --frames 10485760 --calls 10 --warmup 2 --sync --timed > "$OUT/cur.log" 2>&1 || exit 1
grep Mpackets "$OUT/cur.log"
