#!/usr/bin/env python3
"""Per-kernel stats and a slice of the kernel timeline from a rocprofv3 --kernel-trace directory."""
import collections
import glob
import sqlite3
import statistics
import sys

d = sys.argv[1]
first, count = (int(sys.argv[2]), int(sys.argv[3])) if len(sys.argv) > 3 else (40, 40)
db = glob.glob(d + "/**/*.db", recursive=True)[0]
rows = sorted(sqlite3.connect(db).execute("select name,start,end from kernels"), key=lambda r: r[1])
acc = collections.defaultdict(list)
for name, s, e in rows:
    acc[name[:60]].append((e - s) / 1e3)
for k, v in sorted(acc.items(), key=lambda kv: -sum(kv[1]))[:10]:
    print("%-60s %4d %8.1f %8.1f" % (k, len(v), sum(v) / len(v), statistics.median(v)))
seq = [(n[:24], s, e) for n, s, e in rows if "k_parse_seg" in n or "k_flow" in n]
t0 = None
for n, s, e in seq[first:first + count]:
    t0 = t0 or s
    print("%-24s %9.1f %9.1f %7.1f" % (n, (s - t0) / 1e3, (e - t0) / 1e3, (e - s) / 1e3))
