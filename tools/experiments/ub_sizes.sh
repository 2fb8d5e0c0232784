#!/bin/bash
# GPU box: ubench_ws at several batch sizes (frames), to separate fixed costs from throughput.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
V=${V:-8_3}
for n in ${SIZES:-262144 1048576 4194304}; do
  echo "== n=$n"
  timeout -k 10 120 tools/ubench_ws_$V ${CFG:-2} $n ${ROT:-8} ${ITERS:-100} > gpurun_out/ubs_$n.log 2>&1 || { echo "rc=$?"; tail gpurun_out/ubs_$n.log; exit 1; }
  grep '"variant"' gpurun_out/ubs_$n.log
done
