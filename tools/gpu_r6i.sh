#!/bin/bash
# GPU box, round-6 closing pass at HEAD: the whole -m gpu suite, smoke(), the default bench line
set -u
cd "${GRAFT_REPO_ROOT}"
OUT=gpurun_out/${RUN:-r6i}; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -v --timeout 180 --timeout-method thread > $OUT/gpu_tests.txt 2>&1 || { tail -40 $OUT/gpu_tests.txt; exit 1; }
tail -3 $OUT/gpu_tests.txt
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.txt 2>&1 || { tail -20 $OUT/smoke.txt; exit 1; }
tail -3 $OUT/smoke.txt
timeout -k 10 400 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
tail -c 300 $OUT/bench.json
