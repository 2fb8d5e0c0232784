#!/bin/bash
# Growth + pipelined-bucketing check: the table GPU tests, then the C4 pipelined trace.
set -u
cd "${GRAFT_REPO_ROOT}"; R=$(pwd); export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_grow.py tests/test_gpu_async.py tests/test_gpu_history.py tests/test_gpu_parity.py tests/test_gpu_compact.py tests/test_sessions_filter.py -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/grow_tests.log 2>&1
rc=$?; grep -E "PASS|FAIL|ERROR|passed|failed" gpurun_out/grow_tests.log | tail -40; [ $rc -eq 0 ] || exit $rc
D=$R/gpurun_out/c4pipe; rm -rf $D; mkdir -p $D
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D -o run -- python3 $R/bench.py --config 4 --steps 20 --warmup 3 --no-cpu-baseline --no-host --no-imix --no-other-mode > $D/bench.json 2> $D/bench.err || { grep -v "^[WIE]20" $D/bench.err | tail -5; exit 1; }
cd $R
python3 tools/timeline.py $D 60 30
python3 -c "import json;d=json.load(open('$D/bench.json'));print(d['value'], d['extra']['c4_stages']['flow_update_ms'], d['extra']['c4_sync'])"
