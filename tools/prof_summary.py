#!/usr/bin/env python3
"""Summarise rocprofv3 outputs (rocpd SQLite) of tools/gpu_profile.sh into profiles/.

  --trace DIR  : kernel-trace --stats run  -> per-kernel stats CSV (calls, total/avg/min/max us)
  --fetch DIR / --write DIR : separate --pmc FETCH_SIZE / WRITE_SIZE runs -> per-launch HBM bytes
                 of the parse kernel, raw and with the gfx950 correction of
                 /opt/skills/guides/MI355X_MICROARCH.md (HBM section: FETCH_SIZE reports 1/2 of
                 the bytes of wide 16-B-per-lane streaming reads -> x2; WRITE_SIZE exact for
                 16-B-per-lane stores).  FETCH_SIZE / WRITE_SIZE are in KiB.
Usage: python3 tools/prof_summary.py --tag r01_c2 --trace ... --fetch ... --write ... [--config 2]
"""
import argparse
import glob
import json
import os
import sqlite3
import statistics

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PARSE_KERNEL = "k_parse_seg"


def db_of(d):
    dbs = glob.glob(os.path.join(d, "**", "*.db"), recursive=True)
    if not dbs:
        raise SystemExit("no rocpd database under %s" % d)
    return sqlite3.connect(dbs[0])


def kernel_stats(d):
    c = db_of(d)
    rows = {}
    for name, dur in c.execute("select name, duration from kernels"):
        rows.setdefault(name, []).append(dur / 1e3)  # ns -> us
    tot_all = sum(sum(v) for v in rows.values())
    out = []
    for name, v in sorted(rows.items(), key=lambda kv: -sum(kv[1])):
        out.append(dict(name=name, calls=len(v), total_us=round(sum(v), 3), avg_us=round(sum(v) / len(v), 3),
                        min_us=round(min(v), 3), max_us=round(max(v), 3),
                        median_us=round(statistics.median(v), 3), pct=round(100.0 * sum(v) / tot_all, 2)))
    return out


def dispatches(d, sub):
    """Every dispatch of the kernels whose name contains `sub`, in start order: (name, us)."""
    c = db_of(d)
    return [(n, dur / 1e3) for n, dur, _ in
            c.execute("select name, duration, start from kernels order by start") if sub in n]


def counter(d, name):
    c = db_of(d)
    vals = [v for k, cn, v in c.execute("select kernel_name, counter_name, value from counters_collection")
            if PARSE_KERNEL in k and cn == name]
    if not vals:
        raise SystemExit("no %s samples for %s in %s" % (name, PARSE_KERNEL, d))
    # drop the first (cold) launches of each batch buffer: median is robust
    return statistics.median(vals), len(vals)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tag", required=True)
    ap.add_argument("--config", default="2")
    ap.add_argument("--trace")
    ap.add_argument("--fetch")
    ap.add_argument("--write")
    ap.add_argument("--kernel", default=None, help="substring of the dominant kernel's name (default k_parse_seg)")
    ap.add_argument("--algo-bytes", type=float, default=None, help="algorithmic bytes per launch (bench line)")
    ap.add_argument("--bpl", type=int, default=1, help="batches per launch of the profiled bench run")
    ap.add_argument("--key", default=None, help="pmc_traffic.json key (default: --config)")
    ap.add_argument("--dispatch-kernel", default=None,
                    help="with --trace: also write every dispatch of the kernels matching this substring")
    a = ap.parse_args()
    global PARSE_KERNEL
    if a.kernel:
        PARSE_KERNEL = a.kernel
    os.makedirs(os.path.join(ROOT, "profiles"), exist_ok=True)
    if a.trace:
        st = kernel_stats(a.trace)
        p = os.path.join(ROOT, "profiles", "%s_kernel_stats.csv" % a.tag)
        with open(p, "w") as f:
            f.write("Name,Calls,TotalDurationUs,AverageUs,MedianUs,MinUs,MaxUs,Percentage\n")
            for r in st:
                f.write('"%s",%d,%.3f,%.3f,%.3f,%.3f,%.3f,%.2f\n' % (r["name"], r["calls"], r["total_us"], r["avg_us"],
                                                                     r["median_us"], r["min_us"], r["max_us"], r["pct"]))
        print("wrote", p)
        for r in st[:5]:
            print(r)
        if a.dispatch_kernel:
            p = os.path.join(ROOT, "profiles", "%s_dispatches.csv" % a.tag)
            with open(p, "w") as f:
                f.write("Index,Name,DurationUs\n")
                for i, (n, us) in enumerate(dispatches(a.trace, a.dispatch_kernel)):
                    f.write('%d,"%s",%.3f\n' % (i, n, us))
            print("wrote", p)
    if a.fetch and a.write:
        fkb, nf = counter(a.fetch, "FETCH_SIZE")
        wkb, nw = counter(a.write, "WRITE_SIZE")
        fetch_raw = fkb * 1024.0
        write_raw = wkb * 1024.0
        fetch_corr = 2.0 * fetch_raw
        hbm = fetch_corr + write_raw
        p = os.path.join(ROOT, "profiles", "pmc_traffic.json")
        try:
            d = json.load(open(p))
        except (OSError, ValueError):
            d = {}
        d[a.key or str(a.config)] = dict(
            tag=a.tag, kernel=PARSE_KERNEL, launches_fetch=nf, launches_write=nw,
            fetch_size_kib_median=fkb, write_size_kib_median=wkb,
            fetch_bytes_raw=fetch_raw, fetch_bytes_corrected_x2=fetch_corr, write_bytes=write_raw,
            hbm_bytes_per_launch=hbm, batches_per_launch=a.bpl, hbm_bytes_per_batch=hbm / a.bpl,
            algo_bytes_per_launch=a.algo_bytes,
            note=("separate --pmc passes; FETCH_SIZE doubled per MI355X_MICROARCH.md (gfx950 reports 1/2 of "
                  "16-B-per-lane streaming reads); our header loads are 16-B per lane but unaligned and "
                  "overlapping, so the x2 is an upper estimate; Infinity-Cache hits are counted too"))
        with open(p, "w") as f:
            json.dump(d, f, indent=1, sort_keys=True)
        print("wrote", p, d[a.key or str(a.config)])


if __name__ == "__main__":
    main()
