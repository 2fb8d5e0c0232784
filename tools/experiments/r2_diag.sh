#!/bin/bash
# Kernel-trace profile of a small diagnostic script (argument: the script under tools/).
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export TMPDIR=/tmp
S=${1:-diag_host.py}
rm -rf gpurun_out/diag_prof
cd /tmp && timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/diag_prof -o run -- python3 $GRAFT_REPO_ROOT/tools/$S > $GRAFT_REPO_ROOT/gpurun_out/diag_prof.log 2>&1 || { tail -5 $GRAFT_REPO_ROOT/gpurun_out/diag_prof.log; exit 1; }
grep -v "^[WIE]2026" $GRAFT_REPO_ROOT/gpurun_out/diag_prof.log | tail -20
python3 - <<'PY'
import glob, os, sqlite3
root = os.environ["GRAFT_REPO_ROOT"] + "/gpurun_out/diag_prof"
db = glob.glob(root + "/**/*.db", recursive=True)[0]
c = sqlite3.connect(db)
rows = {}
for name, dur in c.execute("select name, duration from kernels"):
    rows.setdefault(name[:90], []).append(dur / 1e3)
for k, v in sorted(rows.items(), key=lambda kv: -sum(kv[1])):
    v.sort()
    print("%-90s %5d avg %9.2f med %9.2f min %9.2f" % (k, len(v), sum(v) / len(v), v[len(v) // 2], v[0]))
PY
