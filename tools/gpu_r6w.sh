#!/bin/bash
# Timed C4 pipelined call A/B: product vs variants (VARS), timed tests first, then an async kernel trace
set -u
cd "${GRAFT_REPO_ROOT}"
R=$(pwd); OUT=$R/gpurun_out/${RUN:-r6w}; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_timed.py -x -q --timeout 120 ${TESTS_K:-} --timeout-method thread > "$OUT/timed_tests.txt" 2>&1 || { tail -30 "$OUT/timed_tests.txt"; exit 1; }
tail -2 "$OUT/timed_tests.txt"
for rep in 1 2; do
for v in ${VARS:-prod nt}; do
  if [ $v = prod ]; then L=""; else L="$R/flodbadd_amd/build/var_$v.so"; fi
  FLODBADD_GPU_LIB=$L timeout -k 10 120 python3 tools/c4_small_calls.py --frames 10485760 --calls 20 --warmup 3 --timed > "$OUT/c4t_$v.log" 2>&1 || { cat "$OUT/c4t_$v.log"; exit 1; }
  echo "$rep $v $(cat $OUT/c4t_$v.log)"
done
done
cd /tmp
timeout -k 10 180 rocprofv3 --kernel-trace -d "$OUT/tasync" -o run -- python3 "$R/tools/c4_small_calls.py" --frames 10485760 --calls 10 --warmup 2 --timed > "$OUT/tasync.log" 2>&1 || exit 1
