#!/bin/bash
# timing-only K2 ablations at 1M-frame C4 calls (one stream): noslice (the 64-KB slice and ordered
# fields not loaded: LDS zero-filled), nowb (no write-back of touched slots); product beside them
set -u
cd "${GRAFT_REPO_ROOT}"
R=$(pwd); OUT=$R/gpurun_out/r6t; mkdir -p "$OUT"; export TMPDIR=/tmp
cd /tmp
for v in cur noslice; do
  L=$R/flodbadd_amd/build/var_$v.so; [ $v = cur ] && L=$R/flodbadd_amd/libflodbadd_gpu.so
  FLODBADD_GPU_LIB=$L timeout -k 10 180 rocprofv3 --kernel-trace --stats -d "$OUT/$v" -o run -- python3 "$R/tools/c4_small_calls.py" --frames 1048576 --calls 100 --warmup 10 --sync > "$OUT/$v.log" 2>&1 || exit 1
done
