#!/bin/bash
# K2 cost split (uniform C4, one-stream): kernel trace of the product library and timing-only
# variants (local gather = records from a cache-resident window; no slice I/O).
set -u
cd "${GRAFT_REPO_ROOT}"; R=$(pwd); export TMPDIR=/tmp
for v in ${VARS:-product lg nsio lgnsio}; do
  L=""; [ "$v" != product ] && L=$R/flodbadd_amd/build/var_$v.so
  rm -rf $R/gpurun_out/k2p_$v; mkdir -p $R/gpurun_out/k2p_$v
  cd /tmp
  FB_BENCH_ABLATION=1 FLODBADD_GPU_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/k2p_$v -o run -- python3 $R/bench.py --config 4 --c4-sync --steps 10 --warmup 2 --no-cpu-baseline --no-host --no-imix --no-other-mode > $R/gpurun_out/k2p_$v/bench.log 2>&1 || { tail -5 $R/gpurun_out/k2p_$v/bench.log; exit 1; }
  cd $R
  echo "== $v"
  python3 - $R/gpurun_out/k2p_$v <<'PY'
import sqlite3, glob, collections, sys, statistics
db = glob.glob(sys.argv[1] + "/**/*.db", recursive=True)[0]
acc = collections.defaultdict(list)
for name, s, e in sqlite3.connect(db).execute("select name,start,end from kernels"):
    acc[name[:60]].append((e - s) / 1e3)
for k, v in sorted(acc.items(), key=lambda kv: -sum(kv[1]))[:8]:
    print("%-60s %4d %8.1f %8.1f" % (k, len(v), sum(v) / len(v), statistics.median(v)))
PY
done
