"""What ran beside a kernel: for every launch of the kernels matching NAME in a rocprofv3
kernel-trace database, the kernels of OTHER streams that overlapped it in time and for how
long; summed per overlapping kernel, plus the launch durations split by whether anything
overlapped.  Used to attribute the in-loop slowdown of a kernel (e.g. k_gae_1p_seg: ~40 us
isolated, ~150 us inside the update loop) to the side-stream Fisher-Yates / J-expansion
passes it shares the GPU with.

    python scripts/kt_overlap.py KT.db NAME [--top 10]
"""
import argparse
import sqlite3
from collections import defaultdict


def short(name, n=60):
    name = name.replace("bppo::", "")
    return name if len(name) <= n else name[:n - 3] + "..."


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("name")
    ap.add_argument("--top", type=int, default=10)
    a = ap.parse_args()
    db = sqlite3.connect(a.db)
    rows = db.execute("select name, start, end, stream_id, queue_id from kernels order by start").fetchall()
    tgt = [r for r in rows if a.name in r[0]]
    if not tgt:
        raise SystemExit(f"no kernel matching {a.name}")
    ov_time = defaultdict(float)        # overlapping kernel -> summed overlap (us)
    ov_launch = defaultdict(int)        # overlapping kernel -> target launches it overlapped
    alone, shared = [], []
    for t in tgt:
        t0, t1, key = t[1], t[2], (t[3], t[4])
        seen = set()
        cover = 0.0
        for r in rows:
            if r[1] >= t1:
                break
            if r[2] <= t0 or (r[3], r[4]) == key:
                continue
            o = (min(t1, r[2]) - max(t0, r[1])) / 1e3
            if o <= 0:
                continue
            n = short(r[0])
            ov_time[n] += o
            cover += o
            if n not in seen:
                ov_launch[n] += 1
                seen.add(n)
        (shared if cover > 0 else alone).append((t1 - t0) / 1e3)
    dur = [(t[2] - t[1]) / 1e3 for t in tgt]
    print(f"# {a.name}: {len(tgt)} launches, avg {sum(dur) / len(dur):.1f} us (min {min(dur):.1f}, max {max(dur):.1f})")
    if alone:
        print(f"#   with nothing beside it: {len(alone)} launches, avg {sum(alone) / len(alone):.1f} us")
    if shared:
        print(f"#   beside other-stream kernels: {len(shared)} launches, avg {sum(shared) / len(shared):.1f} us")
    print("# overlapping kernel (other streams): launches overlapped, summed overlap us")
    for n, v in sorted(ov_time.items(), key=lambda kv: -kv[1])[:a.top]:
        print(f"  {n:62s} {ov_launch[n]:5d} {v:10.1f}")


if __name__ == "__main__":
    main()
