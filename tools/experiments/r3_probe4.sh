#!/bin/bash
# gather microbenchmark (fixed); kernel trace of the pipelined C4 line (overlapped durations)
set -u
cd "${GRAFT_REPO_ROOT}"; R=$(pwd); export TMPDIR=/tmp
timeout -k 10 120 ./tools/ubench_gather 10485760 10 || exit 1
D=$R/gpurun_out/c4pipe; rm -rf $D; mkdir -p $D
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D -o run -- python3 $R/bench.py --config 4 --steps 20 --warmup 3 --no-cpu-baseline --no-host --no-imix --no-other-mode > $D/bench.json 2> $D/bench.err || { grep -v "^[WIE]20" $D/bench.err | tail -5; exit 1; }
cd $R
python3 - $D <<'PY'
import sqlite3, glob, collections, sys, statistics
db = glob.glob(sys.argv[1] + "/**/*.db", recursive=True)[0]
rows = sorted(sqlite3.connect(db).execute("select name,start,end from kernels"), key=lambda r: r[1])
acc = collections.defaultdict(list)
for name, s, e in rows:
    acc[name[:60]].append((e - s) / 1e3)
for k, v in sorted(acc.items(), key=lambda kv: -sum(kv[1]))[:8]:
    print("%-60s %4d %8.1f %8.1f" % (k, len(v), sum(v) / len(v), statistics.median(v)))
# timeline of the first timed steps: parse / K1 / K2 start-end relative
t0 = None
seq = [(n[:20], s, e) for n, s, e in rows if "k_parse_seg" in n or "k_flow" in n]
for n, s, e in seq[40:80]:
    t0 = t0 or s
    print("%-20s %9.1f %9.1f %7.1f" % (n, (s - t0) / 1e3, (e - t0) / 1e3, (e - s) / 1e3))
PY
python3 -c "import json;d=json.load(open('$D/bench.json'));print(d['value'])"
