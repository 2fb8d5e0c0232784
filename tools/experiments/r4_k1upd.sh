#!/bin/bash
# Round 4: the pipelined call's bucketing (K1, K1c) on the update stream instead of the parse
# stream (FB_K1_ON_UPD=1, an experiment knob read at fb_create) -- interleaved C4 pipelined
# table-only lines (uniform, Zipf(1.1)), kernel traces of both, and the pipelined-path tests with it.
# The knob lives in commit d16e88f (reverted in 4c798ca).
set -u
cd "${GRAFT_REPO_ROOT}"
R=$(pwd); OUT=$R/gpurun_out/r4ku; rm -rf "$OUT"; mkdir -p "$OUT"; export TMPDIR=/tmp
step() { echo "== $(date +%T) $1" >&2; shift; "$@"; rc=$?; echo "rc=$rc" >&2; [ $rc -eq 0 ] || exit $rc; }
X="--no-cpu-baseline --no-host --no-imix --no-other-mode --no-single-launch --no-copy-ref --table-only"
for rep in 1 2 3; do
  for v in 0 1; do
    for z in "" "--zipf 1.1"; do
      f=$OUT/pipe_k${v}_${rep}${z:+z}.json
      step pipe env FB_K1_ON_UPD=$v timeout -k 10 300 python3 bench.py --config 4 $z --steps 20 --warmup 3 $X > "$f" 2> "$f.err"
      python3 -c "import json; d=json.loads(open('$f').readline()); print('k1_on_upd=$v rep $rep zipf=${z:+1}', d['value'], d['ms_per_step'])"
    done
  done
done
cd /tmp
for v in 0 1; do
  step tr_$v env FB_K1_ON_UPD=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/tr_$v" -o run -- python3 "$R/bench.py" --config 4 --steps 10 --warmup 2 $X > "$OUT/tr_$v.json" 2> "$OUT/tr_$v.err"
done
cd "$R"
step tests env FB_K1_ON_UPD=1 timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "async or zipf or hot or history or grow or c4 or combine or pipelined" > "$OUT/tests.log" 2>&1
tail -n 1 "$OUT/tests.log"
