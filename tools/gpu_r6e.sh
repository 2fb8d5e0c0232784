#!/bin/bash
# round 6: default bench line (incl. c4_zipf / c4_1m / c4_timed), then the one-box --gpus 2 rehearsal
# of the C5 line over gloo (two ranks on GPU 0: conservation + the routed table == the merged table)
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/r6e
timeout -k 10 400 python bench.py --steps 20 --warmup 20 > gpurun_out/r6e/bench.json 2> gpurun_out/r6e/bench.err || { tail -20 gpurun_out/r6e/bench.err; exit 1; }
tail -c 300 gpurun_out/r6e/bench.json
FB_C5_BACKEND=gloo timeout -k 10 400 python bench.py --gpus 2 --steps 20 --warmup 10 --no-cpu-baseline --no-other-mode --no-host --no-single-launch --no-imix --no-c4 --c5-frames 4194304 > gpurun_out/r6e/gpus2.json 2> gpurun_out/r6e/gpus2.err
rc=$?
tail -c 1500 gpurun_out/r6e/gpus2.json; echo "rc=$rc"; tail -5 gpurun_out/r6e/gpus2.err
