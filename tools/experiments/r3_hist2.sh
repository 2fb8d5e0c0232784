#!/bin/bash
# History GPU tests + kernel timing of the product and variants (VARS).
set -u
cd "${GRAFT_REPO_ROOT}"; R=$(pwd); export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_history.py tests/test_gpu_async.py tests/test_gpu_grow.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/hist_tests.log 2>&1
rc=$?; tail -3 gpurun_out/hist_tests.log; [ $rc -eq 0 ] || exit $rc
for v in ${VARS:-product}; do
  L=""; [ "$v" != product ] && L=$R/flodbadd_amd/build/var_$v.so
  rm -rf $R/gpurun_out/hv_$v; mkdir -p $R/gpurun_out/hv_$v
  cd /tmp
  FLODBADD_GPU_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/hv_$v -o run -- python3 $R/bench.py --config 4 --c4-sync --steps 6 --warmup 2 --no-cpu-baseline --no-host --no-imix --no-other-mode > $R/gpurun_out/hv_$v/bench.json 2> $R/gpurun_out/hv_$v/bench.err || { tail -5 $R/gpurun_out/hv_$v/bench.err; exit 1; }
  cd $R
  echo "== $v"
  python3 - $R/gpurun_out/hv_$v <<'PY'
import sqlite3, glob, collections, sys, json
db = glob.glob(sys.argv[1] + "/**/*.db", recursive=True)[0]
acc = collections.defaultdict(list)
for name, s, e in sqlite3.connect(db).execute("select name,start,end from kernels"):
    if "hist" in name: acc[name[:40]].append((e - s) / 1e3)
for k, v in acc.items(): print("%-40s %3d %8.1f" % (k, len(v), sum(v) / len(v)))
d = json.load(open(sys.argv[1] + "/bench.json"))
print("history_ms", d["extra"]["c4_stages"]["history_ms"])
PY
done
