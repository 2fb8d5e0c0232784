#!/bin/bash
# C4 one-stream run (table-only unless C4REC=1) under a kernel trace: per-kernel averages.
set -u
cd "${GRAFT_REPO_ROOT}"; R=$(pwd); export TMPDIR=/tmp; mkdir -p gpurun_out
L=""; [ -n "${VAR:-}" ] && L="$R/flodbadd_amd/build/var_$VAR.so"
T="--table-only"; [ -n "${C4REC:-}" ] && T=""
D=$R/gpurun_out/c4prof; rm -rf $D; mkdir -p $D
cd /tmp
FB_BENCH_ABLATION=1 FLODBADD_GPU_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D -o run -- python3 $R/bench.py --config 4 --c4-sync --steps 20 --warmup 3 --no-cpu-baseline --no-host --no-imix --no-other-mode $T > $D/bench.json 2> $D/bench.err || { grep -v "^[WIE]20" $D/bench.err | tail -5; exit 1; }
cd $R
f=$(find $D -name "*kernel_stats.csv" | head -1); python3 -c "
import csv,sys
rows=list(csv.DictReader(open('$f')))
for r in sorted(rows,key=lambda r:-float(r['TotalDurationNs']))[:14]:
    print('%-60s %6s %10.1f us' % (r['Name'][:60], r['Calls'], float(r['AverageNs'])/1e3))
"
