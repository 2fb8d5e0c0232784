#!/bin/bash
# GPU box: closing pass (-m gpu suite, smoke, default bench line) + an async timed-C4 kernel trace
set -u
cd "${GRAFT_REPO_ROOT}"
R=$(pwd); OUT=$R/gpurun_out/${RUN:-r6v}; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -v --timeout 180 --timeout-method thread > $OUT/gpu_tests.txt 2>&1 || { tail -40 $OUT/gpu_tests.txt; exit 1; }
tail -3 $OUT/gpu_tests.txt
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.txt 2>&1 || { tail -20 $OUT/smoke.txt; exit 1; }
tail -3 $OUT/smoke.txt
timeout -k 10 400 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
tail -c 300 $OUT/bench.json
cd /tmp
timeout -k 10 180 rocprofv3 --kernel-trace -d "$OUT/tasync" -o run -- python3 "$R/tools/c4_small_calls.py" --frames 10485760 --calls 10 --warmup 2 --timed > "$OUT/tasync.log" 2>&1 || exit 1
cat "$OUT/tasync.log"
