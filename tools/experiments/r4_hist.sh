#!/bin/bash
# Round 4: the history kernels -- GPU history / parity tests, then the C4 Zipf(1.1) and uniform
# history timing under a kernel trace (one-stream, table-only).
set -u
cd "${GRAFT_REPO_ROOT}"
R=$(pwd); OUT=$R/gpurun_out/r4h; rm -rf "$OUT"; mkdir -p "$OUT"; export TMPDIR=/tmp
step() { echo "== $(date +%T) $1" >&2; shift; "$@"; rc=$?; echo "rc=$rc" >&2; [ $rc -eq 0 ] || exit $rc; }
step tests timeout -k 10 900 python3 -u -m pytest tests/test_gpu_history.py tests/test_gpu_grow.py tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_segmented.py -x -v --timeout 300 --timeout-method thread > "$OUT/tests.log" 2>&1
tail -3 "$OUT/tests.log"
X="--no-cpu-baseline --no-host --no-imix --no-other-mode --no-single-launch"
cd /tmp
step zipf timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/zipf" -o run -- python3 "$R/bench.py" --config 4 --zipf 1.1 --c4-sync --table-only --steps 10 --warmup 2 $X > "$OUT/zipf.json" 2> "$OUT/zipf.err"
step unif timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/unif" -o run -- python3 "$R/bench.py" --config 4 --c4-sync --table-only --steps 10 --warmup 2 $X > "$OUT/unif.json" 2> "$OUT/unif.err"
