#!/bin/bash
# Full GPU suite, then the default bench line (driver's command) under rocprof kernel trace.
set -u
cd "${GRAFT_REPO_ROOT}"; R=$(pwd); export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/full_tests.log 2>&1
rc=$?; tail -3 gpurun_out/full_tests.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error" gpurun_out/full_tests.log | head; exit $rc; }
D=$R/gpurun_out/fullbench; rm -rf $D; mkdir -p $D
timeout -k 10 600 python3 bench.py > $D/bench.json 2> $D/bench.err || { tail -5 $D/bench.err; exit 1; }
python3 -c "
import json; d=json.load(open('$D/bench.json')); e=d['extra']
print(d['value'], d['roofline']['frac'], d['cpu_baseline']['value'])
for k in ('c4','c4_zipf','mode_dense','imix_c3'):
    v=e.get(k); print(k, {kk: v[kk] for kk in list(v)[:12]} if isinstance(v, dict) else v)
"
