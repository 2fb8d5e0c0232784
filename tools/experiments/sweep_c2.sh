#!/bin/bash
# C2 headline A/B over prebuilt library variants (tools/build_variants.sh), interleaved rounds:
# SWEEP_VARIANTS="a b" [SWEEP_ROUNDS="1 2 3"] [STEPS=200] bash tools/experiments/sweep_c2.sh
mkdir -p gpurun_out/sweepc2
set -e
for r in ${SWEEP_ROUNDS:-1 2 3}; do
for v in $SWEEP_VARIANTS; do
  FLODBADD_GPU_LIB=$PWD/flodbadd_amd/build/var_$v.so timeout -k 10 150 python bench.py --steps ${STEPS:-200} --warmup 20 ${ARGS:---no-cpu-baseline --no-host --no-imix --no-other-mode --no-single-launch} > gpurun_out/sweepc2/$v.$r.json 2> gpurun_out/sweepc2/$v.$r.err
  echo "$v $r $(python -c "import json;d=json.loads(open('gpurun_out/sweepc2/$v.$r.json').read().strip().splitlines()[-1]);r=d['roofline'];print(d['value'],r['frac'],r['kernel_ms_per_launch'],d.get('extra',{}).get('imix_c3',{}).get('value'))")"
done
done
