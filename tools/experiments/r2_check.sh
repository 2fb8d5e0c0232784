#!/bin/bash
# GPU tests (all), smoke, then bench lines at the driver's settings and at 200 steps.
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r2_pytest.log 2>&1; rc=$?; tail -5 gpurun_out/r2_pytest.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r2_smoke.log 2>&1 || { tail gpurun_out/r2_smoke.log; exit 1; }
timeout -k 10 240 python bench.py --steps 20 --warmup 5 > gpurun_out/r2_b20.json 2>gpurun_out/r2_b20.err || { tail gpurun_out/r2_b20.err; exit 1; }
timeout -k 10 240 python bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-host > gpurun_out/r2_b200.json 2>gpurun_out/r2_b200.err || { tail gpurun_out/r2_b200.err; exit 1; }
python -c "
import json
for f in ('gpurun_out/r2_b20.json','gpurun_out/r2_b200.json'):
    d=json.load(open(f)); print(f, d['value'], d['roofline']['frac'], d['roofline']['kernel_ms_per_launch'], d['ms_per_step'], {k:v.get('value') for k,v in d.get('extra',{}).items() if isinstance(v,dict)})
"
