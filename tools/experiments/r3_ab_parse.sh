#!/bin/bash
# A/B of parse variants on C2 and C3 (interleaved rounds): FLODBADD_GPU_LIB per variant.
set -u
cd "${GRAFT_REPO_ROOT}"; R=$(pwd); export TMPDIR=/tmp; mkdir -p gpurun_out/ab
for round in 1 2 3; do
  for v in ${VARS:-product}; do
    L=""; [ "$v" != product ] && L=$R/flodbadd_amd/build/var_$v.so
    for cfg in 2 3; do
      FLODBADD_GPU_LIB=$L timeout -k 10 200 python3 bench.py --config $cfg --steps 200 --warmup 20 --no-cpu-baseline --no-c4 --no-host --no-imix --no-other-mode --no-single-launch > gpurun_out/ab/${v}_c${cfg}_$round.json 2> gpurun_out/ab/err.log || { tail -5 gpurun_out/ab/err.log; exit 1; }
      python3 -c "import json; d=json.load(open('gpurun_out/ab/${v}_c${cfg}_$round.json')); print('$round $v c$cfg', d['value'], d['roofline']['frac'])"
    done
  done
done
