#!/bin/bash
# Dense-path GPU tests, then the dense C2/C3 rate: single-pass product vs variants
# (tools/build_variants.sh: twopass = -DFB_DENSE_TWO_PASS), interleaved.
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_dense.py tests/test_gpu_compact.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/dense_pytest.log 2>&1; rc=$?; tail -5 gpurun_out/dense_pytest.log; [ $rc -eq 0 ] || exit $rc
for v in ${DVTEST:-}; do  # variants whose outputs must be checked too
  FLODBADD_GPU_LIB=$(pwd)/flodbadd_amd/build/var_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_dense.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/dense_pytest_$v.log 2>&1; rc=$?; echo "$v: $(tail -1 gpurun_out/dense_pytest_$v.log)"; [ $rc -eq 0 ] || exit $rc
done
X="--mode dense --no-cpu-baseline --no-host --no-other-mode --no-single-launch --no-imix"
for r in 1 2; do
  for v in ${DVARS:-product twopass}; do
    if [ $v = product ]; then L=""; else L="$(pwd)/flodbadd_amd/build/var_$v.so"; fi
    for c in ${DCFGS:-2 3}; do
      FLODBADD_GPU_LIB=$L timeout -k 10 120 python bench.py --config $c --steps 100 --warmup 10 $X > gpurun_out/dab.json 2>gpurun_out/dab.err || { tail gpurun_out/dab.err; exit 1; }
      python -c "import json;d=json.load(open('gpurun_out/dab.json'));print('$v C$c', d['value'], d['roofline']['kernel_ms_per_launch'])"
    done
  done
done
