#!/bin/bash
# Round 5, closing run at HEAD: every GPU test, smoke(), then the driver's default bench line.
set -u
cd "${GRAFT_REPO_ROOT}"
R=$(pwd); OUT=$R/gpurun_out/${RUN_TAG:-r5f}; rm -rf "$OUT"; mkdir -p "$OUT"
step() { echo "== $(date +%T) $1" >&2; shift; "$@"; rc=$?; echo "rc=$rc" >&2; [ $rc -eq 0 ] || exit $rc; }
step tests timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/gputests.log" 2>&1
tail -1 "$OUT/gputests.log"
step smoke timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$OUT/smoke.log" 2>&1
step bench timeout -k 10 600 python3 bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"
python3 -c "import json; d=json.loads(open('$OUT/bench.json').readline()); print(d['value'], d['roofline']['frac'], d['roofline']['stream_copy_GBs'], d['roofline']['frac_of_copy'])"
