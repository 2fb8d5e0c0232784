#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT}"
R=$(pwd); OUT=$R/gpurun_out/${RUN:-r6j}; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_queue.py -x -v --timeout 120 --timeout-method thread -m gpu > "$OUT/tests.log" 2>&1 || { tail -30 "$OUT/tests.log"; exit 1; }
tail -2 "$OUT/tests.log"
cd /tmp
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d "$OUT/qt" -o run -- python3 "$R/tools/queue_table_prof.py" 40 > "$OUT/qt.log" 2>&1 || { tail "$OUT/qt.log"; exit 1; }
grep Mpackets "$OUT/qt.log"
cd "$R" && timeout -k 10 200 python bench.py --steps 50 --no-cpu-baseline --no-imix --no-other-mode --no-host > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail "$OUT/bench.err"; exit 1; }
python -c "import json;d=json.loads(open('$OUT/bench.json').read().splitlines()[-1]);print(d['value'],{k:v.get('value') for k,v in d['extra'].items() if isinstance(v,dict)})"
