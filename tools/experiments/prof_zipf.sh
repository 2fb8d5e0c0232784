# rocprof kernel stats of the C4 Zipf(1.1) one-stream run, per library variant (VARS="a b", prebuilt
# by tools/build_variants.sh; empty: the product build)
set -e
R=$(pwd); export TMPDIR=/tmp
for v in ${VARS:-product}; do
  L=""; [ "$v" != product ] && L=$R/flodbadd_amd/build/var_$v.so
  mkdir -p $R/gpurun_out/profz_$v
  cd /tmp
  FB_BENCH_ABLATION=1 FLODBADD_GPU_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/profz_$v -o run -- python3 $R/bench.py --config 4 --zipf ${ZIPF:-1.1} --c4-sync --steps 10 --warmup 2 --no-cpu-baseline --no-host --no-imix --no-other-mode > $R/gpurun_out/profz_$v/bench.log 2>&1
  cd $R
  echo "== $v"
  python3 - $R/gpurun_out/profz_$v <<'PY'
import sqlite3, glob, collections, sys
db = glob.glob(sys.argv[1] + "/**/*.db", recursive=True)[0]
acc = collections.defaultdict(list)
for name, s, e in sqlite3.connect(db).execute("select name,start,end from kernels"):
    acc[name[:48]].append((e - s) / 1e3)
for k, v in sorted(acc.items(), key=lambda kv: -sum(kv[1]))[:7]:
    print("%-48s %4d %8.1f" % (k, len(v), sum(v) / len(v)))
PY
done
