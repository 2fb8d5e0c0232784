#!/bin/bash
# Timed pass: pair sort over K2's words (time carried as the value, no gather kernel), radix bits A/B;
# timed parity tests first, then the timed C4 call timing per library, then a kernel trace of the product.
set -u
cd "${GRAFT_REPO_ROOT}"
R=$(pwd); OUT=$R/gpurun_out/r6t; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_timed.py -x -q --timeout 120 --timeout-method thread > "$OUT/timed_tests.txt" 2>&1 || { tail -30 "$OUT/timed_tests.txt"; exit 1; }
tail -3 "$OUT/timed_tests.txt"
for v in head b8 prod; do
  if [ $v = prod ]; then L=""; else L="$R/flodbadd_amd/build/var_$v.so"; fi
  FLODBADD_GPU_LIB=$L timeout -k 10 120 python3 tools/c4_small_calls.py --frames 10485760 --calls 20 --warmup 3 --timed > "$OUT/c4t_$v.log" 2>&1 || { cat "$OUT/c4t_$v.log"; exit 1; }
  echo "$v $(cat $OUT/c4t_$v.log)"
done
cd /tmp
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run -- python3 "$R/tools/c4_small_calls.py" --frames 10485760 --calls 10 --warmup 2 --sync --timed > "$OUT/prof.log" 2>&1 || exit 1
cat "$OUT/prof.log"
