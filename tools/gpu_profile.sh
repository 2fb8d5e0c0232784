#!/bin/bash
# One GPU measurement pass (run on the gpurun box): bench line, kernel-trace stats and
# separate PMC passes (FETCH_SIZE / WRITE_SIZE, never combined with tracing domains).
# Every GPU step has its own time limit; the script stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
OUT=$R/gpurun_out/prof
mkdir -p "$OUT"
export TMPDIR=/tmp
CFG=${CFG:-2}
STEPS=${STEPS:-200}
step() { echo "== $*" >&2; "$@"; rc=$?; echo "rc=$rc" >&2; [ $rc -eq 0 ] || exit $rc; }
step timeout -k 10 400 python3 bench.py --config $CFG --steps $STEPS --warmup 20 > "$OUT/bench_c$CFG.json" 2> "$OUT/bench_c$CFG.err"
cat "$OUT/bench_c$CFG.json"
cd /tmp
step timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace_c$CFG" -o run -- python3 "$R/bench.py" --config $CFG --steps 96 --warmup 8 --no-cpu-baseline --no-imix --no-other-mode --no-host --no-single-launch > "$OUT/trace_c$CFG.log" 2>&1
step timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d "$OUT/pmc_fetch_c$CFG" -o run -- python3 "$R/bench.py" --config $CFG --steps 48 --warmup 8 --no-cpu-baseline --no-imix --no-other-mode --no-host --no-single-launch > "$OUT/pmc_fetch_c$CFG.log" 2>&1
step timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d "$OUT/pmc_write_c$CFG" -o run -- python3 "$R/bench.py" --config $CFG --steps 48 --warmup 8 --no-cpu-baseline --no-imix --no-other-mode --no-host --no-single-launch > "$OUT/pmc_write_c$CFG.log" 2>&1
find "$OUT" -name "*.csv" | head -20
