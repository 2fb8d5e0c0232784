#!/bin/bash
# k_time_runs occupancy A/B (launch-bounds waves per EU), timed C4 calls + one-stream kernel traces
set -u
cd "${GRAFT_REPO_ROOT}"
R=$(pwd); OUT=$R/gpurun_out/r6q; mkdir -p "$OUT"; export TMPDIR=/tmp
for rep in 1 2; do
for v in prod w6 w8; do
  if [ $v = prod ]; then L=""; else L="$R/flodbadd_amd/build/var_$v.so"; fi
  FLODBADD_GPU_LIB=$L timeout -k 10 120 python3 tools/c4_small_calls.py --frames 10485760 --calls 20 --warmup 3 --timed > "$OUT/c4t_$v.log" 2>&1 || { cat "$OUT/c4t_$v.log"; exit 1; }
  echo "$rep $v $(cat $OUT/c4t_$v.log)"
done
done
cd /tmp
for v in prod w6 w8; do
  if [ $v = prod ]; then L=""; else L="$R/flodbadd_amd/build/var_$v.so"; fi
  FLODBADD_GPU_LIB=$L timeout -k 10 180 rocprofv3 --kernel-trace -d "$OUT/t_$v" -o run -- python3 "$R/tools/c4_small_calls.py" --frames 10485760 --calls 10 --warmup 2 --timed --sync > "$OUT/t_$v.log" 2>&1 || exit 1
done
