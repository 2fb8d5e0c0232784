#!/bin/bash
# timed tests at HEAD (512-thread tiles), then the one-box C5 rehearsal: two ranks on the box's one GPU
# over gloo (RCCL needs a GPU per rank), the C5 line with its conservation and routed == merged checks
set -u
cd "${GRAFT_REPO_ROOT}"
OUT=gpurun_out/r6n; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_timed.py tests/test_gpu_c5.py -x -q --timeout 120 --timeout-method thread -m gpu > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
FB_C5_BACKEND=gloo timeout -k 10 500 python bench.py --gpus 2 --steps 20 --warmup 5 --no-cpu-baseline --no-imix --no-host --no-other-mode --no-queue > $OUT/gpus2.json 2> $OUT/gpus2.err || { tail -30 $OUT/gpus2.err; exit 1; }
tail -c 1500 $OUT/gpus2.json
