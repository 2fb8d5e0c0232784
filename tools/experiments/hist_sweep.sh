set -e
for v in r11a r11b r11c; do FLODBADD_GPU_LIB=$PWD/flodbadd_amd/build/var_$v.so timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_history.py > gpurun_out/ht_$v.log 2>&1; tail -1 gpurun_out/ht_$v.log; done
SWEEP_VARIANTS="base r8a r11a r11b r11c" bash tools/experiments/sweep_flow.sh
