#!/bin/bash
# Final HEAD: the C2 headline kernel at the driver's command (kernel trace + separate FETCH_SIZE /
# WRITE_SIZE passes) and the timed C4 call's kernels (FETCH_SIZE / WRITE_SIZE).  Each GPU step has its
# own limit; the script stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT}"
R=$(pwd); OUT=$R/gpurun_out/pmcz; rm -rf "$OUT"; mkdir -p "$OUT"; export TMPDIR=/tmp
cd /tmp
B="$R/bench.py --steps 20 --warmup 20 --no-cpu-baseline --no-imix --no-other-mode --no-host --no-single-launch --no-c4 --no-copy-ref"
step() { echo "== $1" >&2; shift; "$@" || { echo "FAILED rc=$?" >&2; exit 1; }; }
step trace_c2 timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$OUT/trace_c2" -o run -- python3 $B > "$OUT/trace_c2.json" 2> "$OUT/trace_c2.err"
step fetch_c2 timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d "$OUT/fetch_c2" -o run -- python3 $B > "$OUT/fetch_c2.json" 2> "$OUT/fetch_c2.err"
step write_c2 timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d "$OUT/write_c2" -o run -- python3 $B > "$OUT/write_c2.json" 2> "$OUT/write_c2.err"
S="$R/tools/c4_small_calls.py --sync --timed --frames 10485760 --calls 10 --warmup 2"
step fetch_t timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d "$OUT/fetch_t" -o run -- python3 $S > "$OUT/fetch_t.log" 2>&1
step write_t timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d "$OUT/write_t" -o run -- python3 $S > "$OUT/write_t.log" 2>&1
tail -c 300 "$OUT/trace_c2.json"
