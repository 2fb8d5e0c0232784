#!/bin/bash
# Round 4: K1 moving the update entries into partition order (FB_K1_UNITS=1) -- GPU tests with it,
# then C4 table-only (one-stream and pipelined, uniform and Zipf(1.1)) with and without, interleaved.
set -u
cd "${GRAFT_REPO_ROOT}"
R=$(pwd); OUT=$R/gpurun_out/r4u; rm -rf "$OUT"; mkdir -p "$OUT"
FB_K1_UNITS=1 timeout -k 10 600 python3 -u -m pytest tests/test_gpu_segmented.py tests/test_gpu_fullsize.py tests/test_gpu_history.py tests/test_gpu_async.py tests/test_gpu_grow.py -x -q --timeout 300 --timeout-method thread > "$OUT/tests.log" 2>&1 || { tail -30 "$OUT/tests.log"; exit 1; }
tail -1 "$OUT/tests.log"
X="--no-cpu-baseline --no-host --no-imix --no-other-mode --no-single-launch --table-only --steps 20 --warmup 3"
for rep in 1 2; do
  for u in 0 1; do
    for z in "" "--zipf 1.1"; do
      FB_K1_UNITS=$u timeout -k 10 200 python3 bench.py --config 4 $z $X > "$OUT/u$u$rep${z:+z}.json" 2> "$OUT/u$u$rep${z:+z}.err" || { tail -3 "$OUT/u$u$rep${z:+z}.err"; exit 1; }
      python3 -c "import json; d=json.loads(open('$OUT/u$u$rep${z:+z}.json').readline()); e=d['extra']; print('units=$u rep=$rep zipf=${z:+1}', d['value'], d['ms_per_step'], 'sync', e['c4_sync']['value'], 'parse', e['c4_stages']['parse_ms'], 'upd', e['c4_stages']['flow_update_ms'])"
    done
  done
done
