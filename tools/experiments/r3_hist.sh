#!/bin/bash
# History without rocPRIM: the history/table GPU tests, then the C4 bench under rocprof (history_ms,
# and the kernel list to confirm no rocprim kernels).
set -u
cd "${GRAFT_REPO_ROOT}"; R=$(pwd); export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_history.py tests/test_gpu_async.py tests/test_gpu_grow.py tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/hist_tests.log 2>&1
rc=$?; grep -E "PASS|FAIL|ERROR|passed|failed|Error|assert" gpurun_out/hist_tests.log | tail -40; [ $rc -eq 0 ] || exit $rc
D=$R/gpurun_out/c4hist; rm -rf $D; mkdir -p $D
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D -o run -- python3 $R/bench.py --config 4 --steps 20 --warmup 3 --no-cpu-baseline --no-host --no-imix --no-other-mode > $D/bench.json 2> $D/bench.err || { grep -v "^[WIE]20" $D/bench.err | tail -5; exit 1; }
cd $R
find $D -name "*kernel_stats.csv" | head -1 | xargs cut -d, -f1-4 | head -30
python3 -c "import json;d=json.load(open('$D/bench.json'));e=d['extra'];print(d['value'], e.get('c4_stages'), e.get('c4_zipf'))"
