#!/bin/bash
# Round 5: queue-fed parse -- tests, then A/B over library variants (tools/build_variants.sh), then
# the per-batch trace (a -DFB_QUEUE_TRACE build).  VARS: variant names (default below).
set -u
cd "${GRAFT_REPO_ROOT}"
R=$(pwd); OUT=$R/gpurun_out/r5qab${TAG:-}; rm -rf "$OUT"; mkdir -p "$OUT"
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_queue.py > "$OUT/qtests.log" 2>&1 || { echo "queue tests failed"; tail -30 "$OUT/qtests.log"; exit 1; }
for v in ${VARS:-product qc8 qc32 qbpc3}; do
  if [ $v = product ]; then L=""; else L="$R/flodbadd_amd/build/var_$v.so"; fi
  FLODBADD_GPU_LIB=$L timeout -k 10 120 python3 tools/experiments/queue_ab.py >> "$OUT/ab.jsonl" 2> "$OUT/$v.err" || { echo "$v failed"; tail -3 "$OUT/$v.err"; exit 1; }
done
for t in ${TRACES:-qtrace}; do
  FLODBADD_GPU_LIB=$R/flodbadd_amd/build/var_$t.so timeout -k 10 120 python3 tools/experiments/queue_trace.py > "$OUT/$t.txt" 2>&1 || { echo "trace $t failed"; tail -5 "$OUT/$t.txt"; exit 1; }
done
grep -h passed "$OUT/qtests.log"; cat "$OUT/ab.jsonl"; grep -h "^{" "$OUT"/qtrace*.txt
