"""Summarise rocprofv3 rocpd databases into the text tables committed under profiles/.

    python scripts/rocpd_summary.py KT.db [--fetch PF.db] [--write PW.db] > profiles/rNN_x.txt

Kernel table: calls, total/avg/min/max duration (us) per kernel, the same
numbers `rocprofv3 --stats` reports.  PMC tables: mean FETCH_SIZE / WRITE_SIZE
per dispatch (KB as reported; on gfx950 FETCH_SIZE counts half the bytes of
wide coalesced reads — MI355X_MICROARCH.md §HBM — so the corrected column doubles it).
"""
import argparse
import sqlite3
from collections import defaultdict


def kernel_stats(path):
    db = sqlite3.connect(path)
    rows = db.execute("select name, duration, start, end from kernels").fetchall()
    agg = defaultdict(list)
    for name, dur, _, _ in rows:
        agg[name].append(dur / 1000.0)
    span = (max(r[3] for r in rows) - min(r[2] for r in rows)) / 1e6 if rows else 0.0
    return agg, span


def pmc(path, counter):
    db = sqlite3.connect(path)
    rows = db.execute("select kernel_name, value from counters_collection where counter_name = ?",
                      (counter,)).fetchall()
    agg = defaultdict(list)
    for name, v in rows:
        agg[name].append(v)
    return agg


def short(name, n=70):
    return name if len(name) <= n else name[:n - 3] + "..."


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("kt")
    ap.add_argument("--fetch")
    ap.add_argument("--write")
    a = ap.parse_args()
    agg, span = kernel_stats(a.kt)
    total = sum(sum(v) for v in agg.values())
    print(f"# kernel trace: {a.kt}")
    print(f"# total kernel time {total / 1000:.3f} ms over a {span:.3f} ms trace span")
    print(f"{'kernel':72s} {'calls':>6s} {'total_us':>12s} {'avg_us':>10s} {'min_us':>10s} {'max_us':>10s} {'pct':>6s}")
    for name, v in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
        s = sum(v)
        print(f"{short(name):72s} {len(v):6d} {s:12.1f} {s / len(v):10.2f} {min(v):10.2f} {max(v):10.2f} "
              f"{100 * s / total:6.2f}")
    for label, path, counter, corr in (("FETCH_SIZE", a.fetch, "FETCH_SIZE", 2.0),
                                       ("WRITE_SIZE", a.write, "WRITE_SIZE", 1.0)):
        if not path:
            continue
        p = pmc(path, counter)
        print(f"\n# {label} per dispatch (KB as reported; corrected = x{corr:g} per gfx950 rule): {path}")
        print(f"{'kernel':72s} {'calls':>6s} {'mean_KB':>12s} {'corrected_MB':>13s}")
        for name, v in sorted(p.items(), key=lambda kv: -sum(kv[1])):
            m = sum(v) / len(v)
            print(f"{short(name):72s} {len(v):6d} {m:12.1f} {m * corr / 1024:13.3f}")


if __name__ == "__main__":
    main()
