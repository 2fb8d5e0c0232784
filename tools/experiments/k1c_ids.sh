# K1c combined-entry ids reserved per workgroup: GPU tests (product build), per-kernel Zipf
# profile and sweep against the previous build (tools/build_variants.sh: ids = this, prev = HEAD)
set -e
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
VARS="ids prev" bash tools/experiments/prof_zipf.sh
ZIPF=1.1 SWEEP_VARIANTS="ids prev" SWEEP_ROUNDS="1 2" bash tools/experiments/sweep_flow.sh
SWEEP_VARIANTS="ids prev" SWEEP_ROUNDS="1" bash tools/experiments/sweep_flow.sh
