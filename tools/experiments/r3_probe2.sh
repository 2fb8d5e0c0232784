#!/bin/bash
# K2 with partition-ordered frames (tools/experiments/k2_local.py) vs the original order, kernel traces; then
# the default bench line at the driver's settings (with the new C4 extra).
set -u
cd "${GRAFT_REPO_ROOT}"; R=$(pwd); export TMPDIR=/tmp
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
  rm -rf $R/gpurun_out/k2l_$o; mkdir -p $R/gpurun_out/k2l_$o
  cd /tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/k2l_$o -o run -- python3 $R/tools/experiments/k2_local.py --order $o -- --config 4 --c4-sync --steps 10 --warmup 2 --no-cpu-baseline --no-host --no-imix --no-other-mode > $R/gpurun_out/k2l_$o/bench.json 2> $R/gpurun_out/k2l_$o/bench.err || { grep -v "^[WIE]20" $R/gpurun_out/k2l_$o/bench.err | tail -5; exit 1; }
  cd $R
  echo "== $o"; summ $R/gpurun_out/k2l_$o
  python3 -c "import json;d=json.load(open('$R/gpurun_out/k2l_$o/bench.json'));print(d['value'],d['extra']['c4_stages']['parse_ms'],d['extra']['c4_stages']['flow_update_ms'])"
done
timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 > gpurun_out/r3_default.json 2> gpurun_out/r3_default.err || { tail -5 gpurun_out/r3_default.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/r3_default.json'));print(d['value'],d['roofline']['frac']);print(json.dumps(d['extra']['c4'])[:1500]);print(d['cpu_baseline'])"
