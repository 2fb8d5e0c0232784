#!/bin/bash
# History kernel cost split: C4 one-stream kernel trace of the product and timing-only variants.
set -u
cd "${GRAFT_REPO_ROOT}"; R=$(pwd); export TMPDIR=/tmp
for v in ${VARS:-product}; do
  L=""; [ "$v" != product ] && L=$R/flodbadd_amd/build/var_$v.so
  rm -rf $R/gpurun_out/hv_$v; mkdir -p $R/gpurun_out/hv_$v
  cd /tmp
  FB_BENCH_ABLATION=1 FLODBADD_GPU_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/hv_$v -o run -- python3 $R/bench.py --config 4 --c4-sync --steps 6 --warmup 2 --no-cpu-baseline --no-host --no-imix --no-other-mode > $R/gpurun_out/hv_$v/bench.log 2>&1 || { tail -5 $R/gpurun_out/hv_$v/bench.log; exit 1; }
  cd $R
  echo "== $v"
  python3 tools/timeline.py $R/gpurun_out/hv_$v 0 0 | grep -E "hist|apply"
done
