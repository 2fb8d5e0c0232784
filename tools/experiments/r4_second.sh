#!/bin/bash
# Round 4, second pass: where the C4 Zipf(1.1) step and its history go (kernel trace of the
# one-stream table-only run), the pipelined table-only C4 step under a trace (K2 beside the parse),
# and the C5 export + merge timing over RCCL at world size 1 (tools/c5_merge_time.py).
set -u
cd "${GRAFT_REPO_ROOT}"
R=$(pwd); OUT=$R/gpurun_out/r4b; rm -rf "$OUT"; mkdir -p "$OUT"; export TMPDIR=/tmp
step() { echo "== $(date +%T) $1" >&2; shift; "$@"; rc=$?; echo "rc=$rc" >&2; [ $rc -eq 0 ] || exit $rc; }
X="--no-cpu-baseline --no-host --no-imix --no-other-mode --no-single-launch"
step merge timeout -k 10 300 python3 tools/c5_merge_time.py > "$OUT/c5_merge_time.log" 2>&1
cat "$OUT/c5_merge_time.log"
cd /tmp
step zipf timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/zipf" -o run -- python3 "$R/bench.py" --config 4 --zipf 1.1 --c4-sync --table-only --steps 10 --warmup 2 $X > "$OUT/zipf.json" 2> "$OUT/zipf.err"
step c4pipe timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/c4pipe" -o run -- python3 "$R/bench.py" --config 4 --table-only --steps 20 --warmup 5 $X > "$OUT/c4pipe.json" 2> "$OUT/c4pipe.err"
step c4sync timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/c4sync" -o run -- python3 "$R/bench.py" --config 4 --c4-sync --table-only --steps 10 --warmup 2 $X > "$OUT/c4sync.json" 2> "$OUT/c4sync.err"
du -sh "$OUT"/* >&2
