#!/bin/bash
# GPU box: C4 update kernels' durations at 10M / 5M / 2.5M frames per batch (same 2^20-flow pool):
# how K1 / K2 scale with the entries per partition (per-entry vs per-workgroup cost).
cd "${GRAFT_REPO_ROOT}"; R=$(pwd); mkdir -p gpurun_out/k2s; export TMPDIR=/tmp
for NP in 10485760 5242880 2621440; do
  rm -rf gpurun_out/k2s/t$NP; cd /tmp
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/k2s/t$NP -o run -- python3 $R/bench.py --config 4 --packets $NP --steps 10 --warmup 2 --no-cpu-baseline --no-other-mode > $R/gpurun_out/k2s/t$NP.log 2>&1 || exit 1
  cd $R
done
