#!/bin/bash
# GPU box, final closing pass at HEAD: -m gpu suite, smoke, default bench line, the one-box two-rank
# rehearsal (both ranks on the one GPU over gloo), an async timed-C4 kernel trace
set -u
cd "${GRAFT_REPO_ROOT}"
R=$(pwd); OUT=$R/gpurun_out/${RUN:-r6z}; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -v --timeout 180 --timeout-method thread > $OUT/gpu_tests.txt 2>&1 || { tail -40 $OUT/gpu_tests.txt; exit 1; }
tail -2 $OUT/gpu_tests.txt
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.txt 2>&1 || { tail -20 $OUT/smoke.txt; exit 1; }
tail -2 $OUT/smoke.txt
timeout -k 10 400 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
tail -c 200 $OUT/bench.json
FB_C5_BACKEND=gloo timeout -k 10 500 python bench.py --gpus 2 > $OUT/bench_gpus2.json 2> $OUT/bench_gpus2.err || { tail -20 $OUT/bench_gpus2.err; exit 1; }
tail -c 300 $OUT/bench_gpus2.json
