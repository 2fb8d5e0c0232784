#!/bin/bash
# Round 4: K1c geometry (keys per table, threads, grid) under C4 Zipf(1.1), one-stream table-only
# kernel traces, product vs variants; then the history / parity tests of the best-looking one.
set -u
cd "${GRAFT_REPO_ROOT}"
R=$(pwd); OUT=$R/gpurun_out/r4kg; rm -rf "$OUT"; mkdir -p "$OUT"; export TMPDIR=/tmp
X="--no-cpu-baseline --no-host --no-imix --no-other-mode --no-single-launch --table-only --c4-sync --zipf 1.1 --config 4 --steps 8 --warmup 2"
cd /tmp
for v in product ${VARS}; do
  L=""; [ "$v" != product ] && L=$R/flodbadd_amd/build/var_$v.so
  FB_BENCH_ABLATION=1 FLODBADD_GPU_LIB=$L timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$OUT/$v" -o run -- python3 "$R/bench.py" $X > "$OUT/$v.json" 2> "$OUT/$v.err" || { echo "$v failed"; tail -3 "$OUT/$v.err"; exit 1; }
  echo "== $v done"
done
cd "$R"
for v in ${TEST_VARS:-}; do
  FLODBADD_GPU_LIB=$R/flodbadd_amd/build/var_$v.so timeout -k 10 600 python3 -u -m pytest tests/test_gpu_history.py tests/test_gpu_parity.py tests/test_gpu_segmented.py -x -q --timeout 300 --timeout-method thread > "$OUT/tests_$v.log" 2>&1 || { tail -20 "$OUT/tests_$v.log"; exit 1; }
  echo "$v tests: $(tail -1 $OUT/tests_$v.log)"
done
