# K2 tag-array probe: GPU tests with the product build, then the tags / notags sweep
set -e
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
SWEEP_VARIANTS="tags notags" SWEEP_ROUNDS="1 2 3" bash tools/experiments/sweep_flow.sh
ZIPF=1.1 SWEEP_VARIANTS="tags notags" SWEEP_ROUNDS="1" bash tools/experiments/sweep_flow.sh
