#!/bin/bash
# C4 with Zipf(1.1) flow popularity as the main line: k_flow_combine knobs (tools/build_variants.sh
# FB_COMB_MIN / FB_COMB_SLOTS) vs the product, interleaved; ZVTEST variants get the history tests first.
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
for v in ${ZVTEST:-}; do
  FLODBADD_GPU_LIB=$(pwd)/flodbadd_amd/build/var_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_history.py tests/test_gpu_parity.py -x -q --timeout 150 --timeout-method thread -p no:cacheprovider > gpurun_out/zipf_$v.log 2>&1; rc=$?; echo "$v: $(tail -1 gpurun_out/zipf_$v.log)"; [ $rc -eq 0 ] || exit $rc
done
X="--config 4 --zipf 1.1 --steps 20 --warmup 4 --no-other-mode --no-cpu-baseline"
for r in 1 2; do
  for v in product ${ZVARS:-}; do
    if [ $v = product ]; then L=""; else L="$(pwd)/flodbadd_amd/build/var_$v.so"; fi
    FLODBADD_GPU_LIB=$L timeout -k 10 200 python bench.py $X > gpurun_out/zab.json 2>gpurun_out/zab.err || { tail gpurun_out/zab.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/zab.json'));e=d['extra'];print('$v', d['value'], e['c4_sync']['value'], e['c4_stages']['flow_update_ms'])"
  done
done
