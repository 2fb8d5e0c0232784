#!/bin/bash
# Round 5: a k_parse_dense launch's duration by the profiler vs the window its blocks run in (first block
# start to last block end, -DFB_DN_TRACE build), same process.
set -u
cd "${GRAFT_REPO_ROOT}"
R=$(pwd); OUT=$R/gpurun_out/r5dw; rm -rf "$OUT"; mkdir -p "$OUT"; export TMPDIR=/tmp
cd /tmp
FLODBADD_GPU_LIB=$R/flodbadd_amd/build/var_dntr.so timeout -k 10 200 rocprofv3 --kernel-trace -d "$OUT/trace" -o run -- python3 "$R/tools/experiments/dense_trace.py" > "$OUT/trace.txt" 2>&1 || { tail -5 "$OUT/trace.txt"; exit 1; }
grep "^{" "$OUT/trace.txt"
python3 "$R/tools/rocpd_summary.py" "$OUT/trace/run_results.db" k_parse_dense | tail -3
python3 - "$OUT/trace/run_results.db" <<'PY'
import sqlite3, sys
rows = [r for r in sqlite3.connect(sys.argv[1]).execute("select name, start, end from kernels order by start") if "k_parse_dense" in r[0]]
n, s, e = rows[-1]
print("last k_parse_dense dispatch: %.2f us" % ((e - s) / 1e3))
PY
