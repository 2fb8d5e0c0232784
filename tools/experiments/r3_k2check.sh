#!/bin/bash
# Table GPU tests (parity, history, combine, grow, async, fullsize), then C4 sync + pipelined traces.
set -u
cd "${GRAFT_REPO_ROOT}"; R=$(pwd); export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_history.py tests/test_gpu_grow.py tests/test_gpu_async.py tests/test_gpu_fullsize.py tests/test_gpu_c5.py tests/test_sessions_filter.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/k2_tests.log 2>&1
rc=$?; tail -3 gpurun_out/k2_tests.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/k2_tests.log | head; exit $rc; }
for mode in sync pipe; do
  D=$R/gpurun_out/k2c_$mode; rm -rf $D; mkdir -p $D
  X=""; [ $mode = sync ] && X="--c4-sync"
  cd /tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D -o run -- python3 $R/bench.py --config 4 $X --steps 20 --warmup 3 --no-cpu-baseline --no-host --no-imix --no-other-mode > $D/bench.json 2> $D/bench.err || { tail -5 $D/bench.err; exit 1; }
  cd $R
  echo "== $mode"; python3 tools/timeline.py $D 0 0 | head -8
  python3 -c "import json;d=json.load(open('$D/bench.json'));print(d['value'], d['extra']['c4_stages']['flow_update_ms'], d['extra']['c4_stages']['history_ms'])"
done
