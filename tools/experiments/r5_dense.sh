#!/bin/bash
# Round 5: dense output -- its GPU tests, the product line (interleaved reps) and a per-tile trace
# (a -DFB_DN_TRACE build).
set -u
cd "${GRAFT_REPO_ROOT}"
R=$(pwd); OUT=$R/gpurun_out/r5dn${TAG:-}; rm -rf "$OUT"; mkdir -p "$OUT"
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_dense.py tests/test_gpu_compact.py > "$OUT/tests.log" 2>&1 || { echo "dense tests failed"; tail -30 "$OUT/tests.log"; exit 1; }
grep -h passed "$OUT/tests.log"
X="--mode dense --steps 200 --warmup 20 --no-c4 --no-imix --no-other-mode --no-single-launch --no-host --no-cpu-baseline"
for rep in 1 2; do
  timeout -k 10 200 python3 bench.py $X > "$OUT/dense.$rep.json" 2> "$OUT/dense.$rep.err" || { tail -3 "$OUT/dense.$rep.err"; exit 1; }
  python3 -c "import json; d=json.loads(open('$OUT/dense.$rep.json').readline()); print('dense', d['value'], d['ms_per_step'])"
  timeout -k 10 200 python3 bench.py --config 3 $X > "$OUT/dense_c3.$rep.json" 2> "$OUT/dense_c3.$rep.err" || { tail -3 "$OUT/dense_c3.$rep.err"; exit 1; }
  python3 -c "import json; d=json.loads(open('$OUT/dense_c3.$rep.json').readline()); print('dense C3', d['value'], d['ms_per_step'])"
done
FLODBADD_GPU_LIB=$R/flodbadd_amd/build/var_dntr.so timeout -k 10 120 python3 tools/experiments/dense_trace.py > "$OUT/trace_c2.txt" 2>&1 || { tail -5 "$OUT/trace_c2.txt"; exit 1; }
cat "$OUT/trace_c2.txt"
