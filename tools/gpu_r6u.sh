#!/bin/bash
# Timed pass sort-config A/B (timing only; the product config passed tests/test_gpu_timed.py in r6t)
set -u
cd "${GRAFT_REPO_ROOT}"
R=$(pwd); OUT=$R/gpurun_out/r6u; mkdir -p "$OUT"; export TMPDIR=/tmp
for rep in 1 2; do
for v in ${VARS:-prod i16 i20 i24 i32}; do
  if [ $v = prod ]; then L=""; else L="$R/flodbadd_amd/build/var_$v.so"; fi
  FLODBADD_GPU_LIB=$L timeout -k 10 120 python3 tools/c4_small_calls.py --frames 10485760 --calls 20 --warmup 3 --timed > "$OUT/c4t_$v.log" 2>&1 || { cat "$OUT/c4t_$v.log"; exit 1; }
  echo "$rep $v $(cat $OUT/c4t_$v.log)"
done
done
