#!/bin/bash
# History kernels: the GPU history tests, then history_ms for C4 uniform and Zipf(1.1) (one stream).
set -u
cd "${GRAFT_REPO_ROOT}"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_history.py tests/test_gpu_async.py -x -q --timeout 100 --timeout-method thread -p no:cacheprovider > gpurun_out/hist_tests.log 2>&1
rc=$?; tail -1 gpurun_out/hist_tests.log; [ $rc -eq 0 ] || exit $rc
for z in "" "--zipf 1.1"; do
  timeout -k 10 200 python3 bench.py --config 4 --c4-sync $z --steps 10 --warmup 2 --no-cpu-baseline --no-host --no-imix --no-other-mode --no-single-launch > gpurun_out/hc.json 2> gpurun_out/hc.err || { tail -5 gpurun_out/hc.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/hc.json'));e=d['extra']['c4_stages'];print('C4 $z', d['value'], 'history_ms', e['history_ms'], e['history_chars'])"
done
