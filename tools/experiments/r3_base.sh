#!/bin/bash
# Round-3 start: the full GPU suite, then the C4 bench line (pipelined + one-stream split).
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r3_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r3_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --config 4 --steps 20 --warmup 5 --no-cpu-baseline --no-host --no-other-mode > gpurun_out/r3_c4.json 2> gpurun_out/r3_c4.err || { tail gpurun_out/r3_c4.err; exit 1; }
tail -c 1500 gpurun_out/r3_c4.json
