#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export TMPDIR=/tmp
true

cd /tmp && timeout -k 10 180 rocprofv3 --kernel-trace --hip-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/diag_prof -o run -- python3 $GRAFT_REPO_ROOT/tools/diag_host.py > $GRAFT_REPO_ROOT/gpurun_out/diag_prof.log 2>&1 || exit 1
find $GRAFT_REPO_ROOT/gpurun_out/diag_prof -name "*stats*"
python3 - <<'PY'
import csv, glob, os
root = os.environ["GRAFT_REPO_ROOT"] + "/gpurun_out/diag_prof"
for f in glob.glob(root + "/**/*kernel_stats.csv", recursive=True) + glob.glob(root + "/**/*hip_api_stats.csv", recursive=True):
    print("==", os.path.basename(f))
    for r in list(csv.DictReader(open(f)))[:14]:
        print(r["Name"][:70], r["Calls"], r["AverageNs"], r["Percentage"])
PY
