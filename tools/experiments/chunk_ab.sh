#!/bin/bash
# K1 bucketing-chunk size variants (tools/build_variants.sh FB_FLOW_CHUNK=...): flow parity tests
# per variant, then the C4 line (pipelined + one-stream split), interleaved with the product.
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
for v in ${CVARS:-ch20k ch24k}; do
  FLODBADD_GPU_LIB=$(pwd)/flodbadd_amd/build/var_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_history.py -x -q --timeout 150 --timeout-method thread -p no:cacheprovider > gpurun_out/chunk_$v.log 2>&1; rc=$?; echo "$v: $(tail -1 gpurun_out/chunk_$v.log)"; [ $rc -eq 0 ] || exit $rc
done
X="--config 4 --steps 20 --warmup 4 --no-other-mode --no-cpu-baseline"
for r in 1 2; do
  for v in product ${CVARS:-ch20k ch24k}; do
    if [ $v = product ]; then L=""; else L="$(pwd)/flodbadd_amd/build/var_$v.so"; fi
    FLODBADD_GPU_LIB=$L timeout -k 10 200 python bench.py $X > gpurun_out/cab.json 2>gpurun_out/cab.err || { tail gpurun_out/cab.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/cab.json'));e=d['extra'];print('$v', d['value'], e['c4_sync']['value'], e['c4_stages']['parse_ms'], e['c4_stages']['flow_update_ms'])"
  done
done
