#!/bin/bash
# C4 change check: the GPU tests that touch the table, then the C4 pipelined line (kernel trace).
set -u
cd "${GRAFT_REPO_ROOT}"; R=$(pwd); export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_async.py tests/test_gpu_history.py tests/test_gpu_segmented.py tests/test_gpu_fullsize.py tests/test_sessions_filter.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/c4check_tests.log 2>&1
rc=$?; tail -3 gpurun_out/c4check_tests.log; [ $rc -eq 0 ] || exit $rc
D=$R/gpurun_out/c4pipe; rm -rf $D; mkdir -p $D
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D -o run -- python3 $R/bench.py --config 4 --steps 20 --warmup 3 --no-cpu-baseline --no-host --no-imix --no-other-mode > $D/bench.json 2> $D/bench.err || { grep -v "^[WIE]20" $D/bench.err | tail -5; exit 1; }
cd $R
python3 tools/timeline.py $D
python3 -c "import json;d=json.load(open('$D/bench.json'));print(d['value'], d['extra']['c4_stages']['flow_update_ms'], d['extra']['c4_sync'])"
