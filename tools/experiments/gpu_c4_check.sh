#!/bin/bash
# GPU check of the C4 path: the GPU tests, then a C4 bench line (each step time-limited).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -5 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --config 4 --steps 40 --warmup 10 --no-cpu-baseline > gpurun_out/c4.json 2> gpurun_out/c4.err
rc=$?; tail -c 1500 gpurun_out/c4.json; exit $rc
