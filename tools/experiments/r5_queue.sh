#!/bin/bash
# Round 5: the resident queue-fed parse -- its GPU tests, then the C2 line's one-batch-per-call
# extras (one launch per batch, and one submit per batch into the queue).
set -u
cd "${GRAFT_REPO_ROOT}"
R=$(pwd); OUT=$R/gpurun_out/${RUN_TAG:-r5q}; rm -rf "$OUT"; mkdir -p "$OUT"
step() { echo "== $(date +%T) $1" >&2; shift; "$@"; rc=$?; echo "rc=$rc" >&2; [ $rc -eq 0 ] || exit $rc; }
step qtests timeout -k 10 300 python3 -u -m pytest tests/test_gpu_queue.py -x -v --timeout 120 --timeout-method thread > "$OUT/qtests.log" 2>&1
tail -3 "$OUT/qtests.log"
step bench timeout -k 10 300 python3 bench.py --steps 64 --warmup 16 --no-cpu-baseline --no-imix --no-other-mode --no-host --no-c4 --no-copy-ref > "$OUT/bench.json" 2> "$OUT/bench.err"
python3 -c "import json; d=json.loads(open('$OUT/bench.json').readline()); e=d['extra']; print(d['value'], e.get('single_batch_launch',{}).get('value'), e.get('single_batch_queue'))"
