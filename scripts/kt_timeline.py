"""Timeline of one update from a rocprofv3 kernel-trace database: per stream, the busy
time and the idle gaps between consecutive kernels, the largest gaps with the kernels
around them.  One update = from a k_cartpole_rollout_mfma start to the next one.

    python scripts/kt_timeline.py KT.db [--update K] [--gaps 12]
"""
import argparse
import sqlite3
from collections import defaultdict


def short(name, n=48):
    name = name.replace("bppo::", "")
    return name if len(name) <= n else name[:n - 3] + "..."


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--update", type=int, default=-2, help="which update (python index over rollouts)")
    ap.add_argument("--gaps", type=int, default=12)
    a = ap.parse_args()
    db = sqlite3.connect(a.db)
    rows = db.execute("select name, start, end, stream_id, queue_id from kernels order by start").fetchall()
    ro = [r[1] for r in rows if "k_cartpole_rollout" in r[0]]
    if len(ro) < 2:
        raise SystemExit("need two rollouts in the trace")
    i = a.update if a.update >= 0 else len(ro) + a.update
    t0, t1 = ro[i], ro[i + 1]
    win = [r for r in rows if t0 <= r[1] < t1]
    print(f"# update {i}: {(t1 - t0) / 1e6:.3f} ms from rollout start to the next rollout start")
    by = defaultdict(list)
    for r in win:
        by[(r[3], r[4])].append(r)
    for key, ks in sorted(by.items(), key=lambda kv: -sum(r[2] - r[1] for r in kv[1])):
        busy = sum(r[2] - r[1] for r in ks) / 1e6
        names = defaultdict(float)
        for r in ks:
            names[short(r[0])] += (r[2] - r[1]) / 1e6
        top = ", ".join(f"{n} {v:.2f}" for n, v in sorted(names.items(), key=lambda kv: -kv[1])[:4])
        print(f"stream {key[0]} queue {key[1]}: {len(ks)} kernels, busy {busy:.3f} ms ({top})")
    # the compute stream: the one with the minibatch kernels
    comp = next(k for k, ks in by.items() if any("k_minibatch" in r[0] for r in ks))
    ks = by[comp]
    gaps = []
    for p, q in zip(ks, ks[1:]):
        g = q[1] - p[2]
        if g > 0:
            gaps.append((g / 1e3, short(p[0]), short(q[0])))
    tot = sum(g[0] for g in gaps) / 1e3
    print(f"# compute stream {comp[0]}: idle {tot:.3f} ms in {len(gaps)} gaps between its kernels; largest:")
    for g, p, q in sorted(gaps, reverse=True)[:a.gaps]:
        print(f"  {g:8.1f} us  after {p:50s} before {q}")


if __name__ == "__main__":
    main()
