#!/bin/bash
# small async batches bucketed on the update stream: async / grow / timed tests, then 1M-frame C4 calls
# product vs bk0 (bucketing on the parse stream, as before), interleaved
set -u
cd "${GRAFT_REPO_ROOT}"
R=$(pwd); OUT=$R/gpurun_out/r6p; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_async.py tests/test_gpu_grow.py tests/test_gpu_timed.py -x -q --timeout 180 --timeout-method thread -m gpu > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for rep in 1 2; do for v in cur bk0; do
  L=$R/flodbadd_amd/build/var_$v.so; [ $v = cur ] && L=$R/flodbadd_amd/libflodbadd_gpu.so
  for fr in 1048576 2097152; do
    echo -n "$v $fr: "; FLODBADD_GPU_LIB=$L timeout -k 10 120 python3 tools/c4_small_calls.py --frames $fr --calls 200 --warmup 20 > $OUT/$v.$fr.$rep.log 2>&1 || { tail $OUT/$v.$fr.$rep.log; exit 1; }
    tail -1 $OUT/$v.$fr.$rep.log
  done
done; done
