#!/bin/bash
# timing-only ablations of k_time_runs (tools/build_variants.sh: noplane, nowrite, nolb) vs the product
set -u
cd "${GRAFT_REPO_ROOT}"
R=$(pwd); OUT=$R/gpurun_out/r6m2; mkdir -p "$OUT"; export TMPDIR=/tmp
cd /tmp
for v in cur t512 i8; do
  L=$R/flodbadd_amd/build/var_$v.so; [ $v = cur ] && L=$R/flodbadd_amd/libflodbadd_gpu.so
  FLODBADD_GPU_LIB=$L timeout -k 10 180 rocprofv3 --kernel-trace --stats -d "$OUT/$v" -o run -- python3 "$R/tools/c4_small_calls.py" --frames 10485760 --calls 10 --warmup 2 --sync --timed > "$OUT/$v.log" 2>&1 || exit 1
done
