# K1c geometry (key-table size, workgroup size, grid): history / async parity per variant, then
# per-kernel Zipf profile and Zipf sweep (tools/build_variants.sh builds)
set -e
mkdir -p gpurun_out
for v in s128 s128j g2k; do
  FLODBADD_GPU_LIB=$PWD/flodbadd_amd/build/var_$v.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_history.py tests/test_gpu_async.py > gpurun_out/t_$v.log 2>&1 || { tail -30 gpurun_out/t_$v.log; exit 1; }
  echo "$v $(tail -1 gpurun_out/t_$v.log)"
done
VARS="base s128 s128j g2k" bash tools/experiments/prof_zipf.sh 2>&1 | grep -E "==|combine"
ZIPF=1.1 SWEEP_VARIANTS="base s128 s128j g2k" SWEEP_ROUNDS="1 2" bash tools/experiments/sweep_flow.sh
