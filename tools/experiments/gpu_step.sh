#!/bin/bash
# Run one GPU validation/measurement pass on the gpurun box.  Each GPU step has its own time
# limit; a crash/abort/timeout (rc >= 2 from pytest, or any signal) stops the script.
# usage: tools/experiments/gpu_step.sh [pytest|smoke|bench|prof|all] ...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
what="${1:-all}"

run_pytest() {
  timeout -k 10 600 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
  rc=$?
  tail -30 gpurun_out/pytest_gpu.log
  echo "pytest rc=$rc"
  # 0 = pass, 1 = test failures: the GPU is fine, keep going; anything else: stop.
  [ $rc -le 1 ]
}
run_smoke() {
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
  rc=$?; cat gpurun_out/smoke.log | tail -5; echo "smoke rc=$rc"; [ $rc -eq 0 ]
}
run_bench() {
  timeout -k 10 600 python bench.py "$@" > gpurun_out/bench.log 2>&1
  rc=$?; tail -5 gpurun_out/bench.log; echo "bench rc=$rc"; [ $rc -eq 0 ]
}

case "$what" in
  pytest) run_pytest ;;
  smoke) run_smoke ;;
  bench) shift; run_bench "$@" ;;
  all) shift; run_pytest && run_smoke && run_bench "$@" ;;
esac
