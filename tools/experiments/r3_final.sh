#!/bin/bash
# Round-3 evidence at HEAD: full GPU suite, the driver's default bench line, the C2 driver command
# under a kernel trace, the C4 (table-only, one stream) trace + FETCH/WRITE passes, a dense C2 trace.
set -u
cd "${GRAFT_REPO_ROOT}"; R=$(pwd); export TMPDIR=/tmp; O=$R/gpurun_out/r3; rm -rf $O; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error" $O/tests.log | head; exit $rc; }
timeout -k 10 600 python3 bench.py > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
python3 -c "
import json; d=json.load(open('$O/bench.json')); e=d['extra']
print('C2', d['value'], d['roofline']['frac'], 'cpu', d['cpu_baseline']['value'])
for k in ('c4','mode_dense','imix_c3'):
    v=e.get(k); print(k, v['value'], v.get('roofline_frac', v.get('roofline', {}).get('frac')))
print('c4_records', e['c4']['c4_records']['value'], 'c4_sync', e['c4']['c4_sync']['value'], e['c4']['c4_stages']['parse_ms'], e['c4']['c4_stages']['flow_update_ms'])
"
bash tools/prof_driver.sh || exit 1
cp -r gpurun_out/profdrv $O/profdrv
NOSQ=1 bash tools/experiments/r3_c4prof.sh || exit 1
cp -r gpurun_out/c4prof $O/c4prof
cd /tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/dense -o run -- python3 $R/bench.py --mode dense --steps 100 --warmup 10 \
  --no-cpu-baseline --no-imix --no-other-mode --no-host --no-single-launch > $O/dense.json 2> $O/dense.err || { tail $O/dense.err; exit 1; }
cd $R; python3 tools/timeline.py $O/dense 0 0 | head -4
