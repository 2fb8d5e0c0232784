#!/bin/bash
# Round 5: grouped update units (k_parse_seg kGroupU + XCD-contiguous K2) in the pipelined C4 call --
# the table tests, then the C4 line with FB_UNIT_GROUP=1 (product) vs 0 (per-segment units), interleaved.
set -u
cd "${GRAFT_REPO_ROOT}"
R=$(pwd); OUT=$R/gpurun_out/r5grp${TAG:-}; rm -rf "$OUT"; mkdir -p "$OUT"
if [ -z "${NOTESTS:-}" ]; then
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_async.py tests/test_gpu_fullsize.py tests/test_gpu_grow.py tests/test_gpu_history.py tests/test_gpu_c5.py > "$OUT/tests.log" 2>&1 || { echo "tests failed"; grep -E "FAILED|Error" "$OUT/tests.log" | head; tail -5 "$OUT/tests.log"; exit 1; }
tail -1 "$OUT/tests.log"
fi
X="--no-cpu-baseline --no-imix --no-other-mode --no-host --no-single-launch --no-queue --no-copy-ref"
for rep in 1 2; do
  for g in 1 0; do
    FB_UNIT_GROUP=$g timeout -k 10 300 python3 bench.py $X > "$OUT/c4_g$g.$rep.json" 2> "$OUT/c4_g$g.$rep.err" || { tail -3 "$OUT/c4_g$g.$rep.err"; exit 1; }
    python3 -c "import json; d=json.loads(open('$OUT/c4_g$g.$rep.json').readline()); c=d['extra']['c4']; print('group=$g', 'c4', c['value'], 'sync', c.get('c4_sync',{}).get('value'), 'stages', c.get('stages', c.get('c4_stages')))"
  done
done
for g in 1 0; do
  FB_UNIT_GROUP=$g timeout -k 10 300 python3 bench.py --config 4 --zipf 1.1 --steps 20 --warmup 4 --no-other-mode --no-cpu-baseline > "$OUT/z_g$g.json" 2> "$OUT/z_g$g.err" || { tail -3 "$OUT/z_g$g.err"; exit 1; }
  python3 -c "import json; d=json.loads(open('$OUT/z_g$g.json').readline()); print('zipf group=$g', d['value'], d['extra'].get('c4_sync',{}).get('value'))"
done
