#!/bin/bash
# GPU box: one rocprofv3 --pmc pass over ubench_ws (counters given in $PMC), summary via sqlite.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd); mkdir -p gpurun_out/pmc; export TMPDIR=/tmp
V=${V:-8_3}; TAG=${TAG:-a}
cd "$R"
timeout -s KILL 120 rocprofv3 --pmc $PMC -d $R/gpurun_out/pmc/$TAG -o run -- $R/tools/ubench_ws_$V 2 1048576 8 20 > $R/gpurun_out/pmc/$TAG.log 2>&1
rc=$?; echo "rc=$rc"; [ $rc -eq 0 ] || { tail -5 $R/gpurun_out/pmc/$TAG.log; exit 1; }
python3 - "$R/gpurun_out/pmc/$TAG" <<'PY'
import glob, sqlite3, sys, statistics, collections
db = glob.glob(sys.argv[1] + "/**/*.db", recursive=True)[0]
c = sqlite3.connect(db)
acc = collections.defaultdict(list)
for k, cn, v in c.execute("select kernel_name, counter_name, value from counters_collection"):
    acc[(k[:60], cn)].append(v)
for (k, cn), v in sorted(acc.items()):
    print("%-60s %-22s n=%4d median=%.6g" % (k, cn, len(v), statistics.median(v)))
PY
