#!/bin/bash
# gather microbenchmark; K2 on partition-ordered frames without the hot-group combine; K2 SQ counters
set -u
cd "${GRAFT_REPO_ROOT}"; R=$(pwd); export TMPDIR=/tmp
timeout -k 10 120 ./tools/ubench_gather 10485760 10 || exit 1
summ() {
python3 - $1 <<'PY'
import sqlite3, glob, collections, sys, statistics
db = glob.glob(sys.argv[1] + "/**/*.db", recursive=True)[0]
acc = collections.defaultdict(list)
for name, s, e in sqlite3.connect(db).execute("select name,start,end from kernels"):
    acc[name[:60]].append((e - s) / 1e3)
for k, v in sorted(acc.items(), key=lambda kv: -sum(kv[1]))[:6]:
    print("%-60s %4d %8.1f %8.1f" % (k, len(v), sum(v) / len(v), statistics.median(v)))
PY
}
for o in partition original; do
  D=$R/gpurun_out/k2n_$o; rm -rf $D; mkdir -p $D
  cd /tmp
  FLODBADD_GPU_LIB=$R/flodbadd_amd/build/var_nocomb.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D -o run -- python3 $R/tools/experiments/k2_local.py --order $o -- --config 4 --c4-sync --steps 10 --warmup 2 --no-cpu-baseline --no-host --no-imix --no-other-mode > $D/bench.json 2> $D/bench.err || { grep -v "^[WIE]20" $D/bench.err | tail -5; exit 1; }
  cd $R
  echo "== nocomb $o"; summ $D
done
KFILT=k_flow_apply ARGS="--config 4 --c4-sync --steps 10 --warmup 2 --no-cpu-baseline --no-host --no-imix --no-other-mode" bash tools/pmc_sq.sh
