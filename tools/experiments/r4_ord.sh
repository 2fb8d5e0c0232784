#!/bin/bash
# Round 4: hot groups placed in record order by K1 -- every GPU test, then the C4 one-stream traces
# (uniform, Zipf(1.1)) and the pipelined table-only lines.
set -u
cd "${GRAFT_REPO_ROOT}"
R=$(pwd); OUT=$R/gpurun_out/r4o; rm -rf "$OUT"; mkdir -p "$OUT"; export TMPDIR=/tmp
step() { echo "== $(date +%T) $1" >&2; shift; "$@"; rc=$?; echo "rc=$rc" >&2; [ $rc -eq 0 ] || exit $rc; }
step tests timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/gputests.log" 2>&1
tail -1 "$OUT/gputests.log"
X="--no-cpu-baseline --no-host --no-imix --no-other-mode --no-single-launch --table-only"
cd /tmp
step zipf timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/zipf" -o run -- python3 "$R/bench.py" --config 4 --zipf 1.1 --c4-sync --steps 10 --warmup 2 $X > "$OUT/zipf.json" 2> "$OUT/zipf.err"
step unif timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/unif" -o run -- python3 "$R/bench.py" --config 4 --c4-sync --steps 10 --warmup 2 $X > "$OUT/unif.json" 2> "$OUT/unif.err"
cd "$R"
for z in "" "--zipf 1.1"; do
  step pipe timeout -k 10 300 python3 bench.py --config 4 $z --steps 20 --warmup 3 $X > "$OUT/pipe${z:+z}.json" 2> "$OUT/pipe${z:+z}.err"
  python3 -c "import json; d=json.loads(open('$OUT/pipe${z:+z}.json').readline()); print('pipelined zipf=${z:+1}', d['value'], d['ms_per_step'])"
done
