#!/bin/bash
# Round 5: two parse blocks per CU in the pipelined call (abpc2, FB_ASYNC_BPC=2) vs the product (one),
# now that K2 starts its heavy partitions first and K1c combines groups of >= 64 records;
# C4 uniform and Zipf(1.1), pipelined table-only, interleaved; the async tests on abpc2.
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
FLODBADD_GPU_LIB=$(pwd)/flodbadd_amd/build/var_abpc2.so timeout -k 10 400 python -u -m pytest tests/test_gpu_async.py tests/test_gpu_fullsize.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/abpc_tests.log 2>&1 || { tail -20 gpurun_out/abpc_tests.log; exit 1; }
tail -1 gpurun_out/abpc_tests.log
for r in 1 2; do
  for v in product abpc2; do
    if [ $v = product ]; then L=""; else L="$(pwd)/flodbadd_amd/build/var_$v.so"; fi
    for z in "" "--zipf 1.1"; do
      FLODBADD_GPU_LIB=$L timeout -k 10 200 python bench.py --config 4 $z --table-only --steps 20 --warmup 4 \
        --no-other-mode --no-cpu-baseline --no-host --no-imix --no-queue --no-copy-ref > gpurun_out/abpc.json 2> gpurun_out/abpc.err || { tail gpurun_out/abpc.err; exit 1; }
      python -c "import json;d=json.load(open('gpurun_out/abpc.json'));e=d['extra'];print('$v', '${z:-uniform}', d['value'], e['c4_sync']['value'], e['c4_stages']['flow_update_ms'])"
    done
  done
done
