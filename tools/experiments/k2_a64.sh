#!/bin/bash
# Experiment (GPU box): K2 with 64-B-aligned record slots (variant a64: records expanded first)
# against the product library, kernel trace of the one-stream C4 bench.  (The FB_K2_ALIGNED64
# experiment code in fb_flow.hip was reverted after the measurement)
cd "${GRAFT_REPO_ROOT}"; R=$(pwd); mkdir -p gpurun_out/a64; export TMPDIR=/tmp
for v in base a64; do
  rm -rf gpurun_out/a64/$v; cd /tmp
  L=""; [ $v = a64 ] && L=$R/flodbadd_amd/build/var_a64.so
  FB_BENCH_ABLATION=1 FLODBADD_GPU_LIB=$L timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/a64/$v -o run -- python3 $R/bench.py --config 4 --c4-sync --steps 10 --warmup 2 --no-cpu-baseline --no-other-mode > $R/gpurun_out/a64/$v.log 2>&1 || exit 1
  cd $R
done
