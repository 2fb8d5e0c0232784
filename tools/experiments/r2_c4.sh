#!/bin/bash
# GPU tests (all), then the C4 bench line and a C4 kernel trace.
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r2_pytest.log 2>&1; rc=$?; tail -5 gpurun_out/r2_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --config 4 --steps 20 --warmup 4 --no-cpu-baseline > gpurun_out/r2_c4.json 2>gpurun_out/r2_c4.err || { tail gpurun_out/r2_c4.err; exit 1; }
python -c "
import json
d=json.load(open('gpurun_out/r2_c4.json')); print(d['value'], d['ms_per_step'], json.dumps(d['extra']['c4_stages'])[:400], d['extra']['c4_zipf'])"
rm -rf gpurun_out/c4prof
cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/c4prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --config 4 --steps 10 --warmup 2 --no-cpu-baseline --no-other-mode > $GRAFT_REPO_ROOT/gpurun_out/c4prof.log 2>&1 || exit 1
