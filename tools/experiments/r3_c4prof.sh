#!/bin/bash
# C4 one-stream run (table-only unless C4REC=1) under a kernel trace, then FETCH_SIZE / WRITE_SIZE
# passes (separate runs) and the SQ counter groups of KFILT (default k_flow_apply).
set -u
cd "${GRAFT_REPO_ROOT}"; R=$(pwd); export TMPDIR=/tmp; mkdir -p gpurun_out
L=""; [ -n "${VAR:-}" ] && L="$R/flodbadd_amd/build/var_$VAR.so"
T="--table-only"; [ -n "${C4REC:-}" ] && T=""
A="--config 4 --c4-sync --no-cpu-baseline --no-host --no-imix --no-other-mode $T"
D=$R/gpurun_out/c4prof; rm -rf $D; mkdir -p $D
cd /tmp
FLODBADD_GPU_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D/trace -o run -- python3 $R/bench.py $A --steps 20 --warmup 3 > $D/bench.json 2> $D/bench.err || { grep -v "^[WIE]20" $D/bench.err | tail -5; exit 1; }
cd $R; python3 tools/timeline.py $D/trace 40 8
[ -n "${NOPMC:-}" ] && exit 0
cd /tmp
for P in FETCH_SIZE WRITE_SIZE; do
  FLODBADD_GPU_LIB=$L timeout -s KILL 120 rocprofv3 --pmc $P -d $D/pmc_$P -o run -- python3 $R/bench.py $A --steps 6 --warmup 2 > $D/pmc_$P.log 2>&1 || { echo "pmc $P failed"; tail -3 $D/pmc_$P.log; exit 1; }
done
cd $R
python3 - $D <<'PY'
import collections, glob, sqlite3, statistics, sys
acc = collections.defaultdict(list)
for d in glob.glob(sys.argv[1] + "/pmc_*"):
    for db in glob.glob(d + "/**/*.db", recursive=True):
        for k, cn, v in sqlite3.connect(db).execute("select kernel_name, counter_name, value from counters_collection"):
            acc[(k[:40], cn)].append(v)
for (k, cn), v in sorted(acc.items()):
    print("%-40s %-12s n=%3d median=%.4g" % (k, cn, len(v), statistics.median(v)))
PY
[ -n "${NOSQ:-}" ] && exit 0
ARGS="$A --steps 6 --warmup 2" KFILT=${KFILT:-k_flow_apply} bash tools/pmc_sq.sh
