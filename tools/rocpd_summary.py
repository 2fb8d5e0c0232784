"""Summary of a rocprofv3 kernel trace stored as a rocpd SQLite database (ROCm 7 writes
<dir>/<name>_results.db when no --output-format is given): per-kernel calls / total / average
(us), and for the top kernel the durations of its dispatches and the idle gaps between them.
Usage: python3 tools/rocpd_summary.py <results.db> [kernel-name-substring]"""
import sqlite3
import sys

import numpy as np

db = sqlite3.connect(sys.argv[1])
print("%-90s %6s %12s %10s" % ("kernel", "calls", "total_us", "avg_us"))
for name, calls, total, avg, _ in db.execute("select * from top_kernels"):
    print("%-90s %6d %12.3f %10.3f" % (name[:90], calls, total, avg))
pat = sys.argv[2] if len(sys.argv) > 2 else None
rows = list(db.execute("select name, start, end from kernels order by start"))
if pat is None:
    pat = next(iter(db.execute("select name from top_kernels limit 1")))[0]
sel = [(s, e) for n, s, e in rows if pat in n]
if sel:
    st = np.array([s for s, _ in sel], dtype=np.float64)
    en = np.array([e for _, e in sel], dtype=np.float64)
    dur = (en - st) / 1e3
    gap = (st[1:] - en[:-1]) / 1e3
    print("\n%s: %d dispatches; duration us median %.3f min %.3f max %.3f" % (pat[:80], len(sel), np.median(dur),
                                                                              dur.min(), dur.max()))
    if len(gap):
        print("gap to the next dispatch (us): median %.3f p10 %.3f p90 %.3f" % (np.median(gap), np.percentile(gap, 10),
                                                                             np.percentile(gap, 90)))
