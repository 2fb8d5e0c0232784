#!/bin/bash
# Round 4: K1c on the update stream (product) vs on the parse stream (var_k1cpar) in the pipelined
# C4 call, uniform and Zipf(1.1), interleaved; then the async / growth / history tests.
set -u
cd "${GRAFT_REPO_ROOT}"
R=$(pwd); OUT=$R/gpurun_out/r4ks; rm -rf "$OUT"; mkdir -p "$OUT"
X="--no-cpu-baseline --no-host --no-imix --no-other-mode --no-single-launch --table-only --config 4 --steps 20 --warmup 3"
for rep in 1 2; do
  for v in product ${VARS:-k1cpar}; do
    L=""; [ "$v" != product ] && L=$R/flodbadd_amd/build/var_$v.so
    for z in "" "--zipf 1.1"; do
      FLODBADD_GPU_LIB=$L timeout -k 10 200 python3 bench.py $z $X > "$OUT/$v$rep${z:+z}.json" 2> "$OUT/$v$rep${z:+z}.err" || { tail -3 "$OUT/$v$rep${z:+z}.err"; exit 1; }
      python3 -c "import json; d=json.loads(open('$OUT/$v$rep${z:+z}.json').readline()); print('$v rep $rep zipf=${z:+1}', d['value'], d['ms_per_step'])"
    done
  done
done
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_async.py tests/test_gpu_grow.py tests/test_gpu_history.py -x -q --timeout 300 --timeout-method thread > "$OUT/tests.log" 2>&1 || { tail -20 "$OUT/tests.log"; exit 1; }
tail -1 "$OUT/tests.log"
