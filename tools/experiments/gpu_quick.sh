#!/bin/bash
# Segmented + full-size GPU tests, then two C2 bench lines (each step time-limited).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_segmented.py tests/test_gpu_fullsize.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/quick.log 2>&1
rc=$?; tail -3 gpurun_out/quick.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-host --no-other-mode --no-single-launch --no-imix > gpurun_out/q$r.json 2>gpurun_out/q$r.err || exit 1
  python -c "import json;d=json.load(open('gpurun_out/q$r.json'));print(d['value'],d['roofline']['frac'],d['roofline']['kernel_ms_per_launch'])"
done
