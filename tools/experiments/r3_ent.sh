#!/bin/bash
# Update entries (fused path) + the store-wave dense kernel: the GPU tests that touch them, the C4
# line with and without SESSION records, and the dense C2 / C3 rates of the product and variants.
set -u
cd "${GRAFT_REPO_ROOT}"; R=$(pwd); export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_async.py tests/test_gpu_dense.py tests/test_gpu_history.py tests/test_gpu_segmented.py tests/test_gpu_fullsize.py tests/test_gpu_grow.py tests/test_sessions_filter.py -m gpu -x -q --timeout 100 --timeout-method thread -p no:cacheprovider > gpurun_out/ent_tests.log 2>&1
rc=$?; tail -3 gpurun_out/ent_tests.log; [ $rc -eq 0 ] || exit $rc
X="--no-cpu-baseline --no-host --no-imix --no-other-mode --no-single-launch"
for r in 1 2; do
  for t in "" "--table-only"; do
    timeout -k 10 200 python3 bench.py --config 4 --steps 20 --warmup 3 $X $t > gpurun_out/c4e.json 2> gpurun_out/c4e.err || { tail -5 gpurun_out/c4e.err; exit 1; }
    python3 -c "import json;d=json.load(open('gpurun_out/c4e.json'));e=d['extra'];print('C4 $t', d['value'], e['c4_stages']['parse_ms'], e['c4_stages']['flow_update_ms'], e['c4_sync']['value'])"
  done
done
for r in 1 2; do
  for v in ${DVARS:-product}; do
    if [ $v = product ]; then L=""; else L="$(pwd)/flodbadd_amd/build/var_$v.so"; fi
    for c in 2 3; do
      FLODBADD_GPU_LIB=$L timeout -k 10 120 python3 bench.py --mode dense --config $c --steps 100 --warmup 10 $X > gpurun_out/dab.json 2>gpurun_out/dab.err || { tail gpurun_out/dab.err; exit 1; }
      python3 -c "import json;d=json.load(open('gpurun_out/dab.json'));print('dense $v C$c', d['value'], d['roofline']['kernel_ms_per_launch'])"
    done
  done
done
