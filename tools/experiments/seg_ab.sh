#!/bin/bash
# Headline C2 (and C3) rate of k_parse_seg variants (tools/build_variants.sh) vs the product,
# interleaved; SVARS names the variants, SVTEST those whose segmented outputs are checked first.
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
for v in ${SVTEST:-}; do
  FLODBADD_GPU_LIB=$(pwd)/flodbadd_amd/build/var_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_segmented.py tests/test_gpu_fullsize.py -x -q --timeout 150 --timeout-method thread -p no:cacheprovider > gpurun_out/seg_$v.log 2>&1; rc=$?; echo "$v: $(tail -1 gpurun_out/seg_$v.log)"; [ $rc -eq 0 ] || exit $rc
done
X="--no-cpu-baseline --no-imix --no-other-mode --no-host --no-single-launch"
for r in 1 2 3; do
  for v in product ${SVARS:-}; do
    if [ $v = product ]; then L=""; else L="$(pwd)/flodbadd_amd/build/var_$v.so"; fi
    for c in ${SCFGS:-2}; do
      FLODBADD_GPU_LIB=$L timeout -k 10 120 python bench.py --config $c --steps 96 --warmup 32 $X > gpurun_out/sab.json 2>gpurun_out/sab.err || { tail gpurun_out/sab.err; exit 1; }
      python -c "import json;d=json.load(open('gpurun_out/sab.json'));r=d['roofline'];print('$v C$c', d['value'], r['kernel_ms_per_launch'], round(r['kernel_ms_per_launch']*1e3/d['config']['batches_per_launch'],2))"
    done
  done
done
