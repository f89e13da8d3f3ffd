"""Per-update timing from a rocprofv3 kernel-trace database of the CfgB bench: for every
update (rollout start to the next rollout start), the span, the compute stream's busy time,
its gaps, the rollout kernel and the minibatch kernels; medians over the updates.

    python scripts/kt_updates.py KT.db [label]
"""
import statistics
import sqlite3
import sys


def main():
    db = sqlite3.connect(sys.argv[1])
    label = sys.argv[2] if len(sys.argv) > 2 else ""
    rows = db.execute("select name, start, end, stream_id from kernels order by start").fetchall()
    ro = [r for r in rows if "rollout_mfma64" in r[0]]
    if len(ro) < 3:
        raise SystemExit("fewer than 3 rollouts in the trace")
    cs = ro[0][3]
    span, busy, roll, mbs, pre = [], [], [], [], []
    for k in range(1, len(ro) - 1):          # skip the warm-up update
        s, nxt = ro[k][1], ro[k + 1][1]
        comp = [x for x in rows if s <= x[1] < nxt and x[3] == cs]
        span.append((nxt - s) / 1e3)
        busy.append(sum(x[2] - x[1] for x in comp) / 1e3)
        roll.append((ro[k][2] - ro[k][1]) / 1e3)
        mbs.append(sum(x[2] - x[1] for x in comp if "minibatch" in x[0]) / 1e3)
        last_mb = max((x[2] for x in comp if "minibatch" in x[0]), default=s)
        pre.append((nxt - last_mb) / 1e3)     # last minibatch end -> next rollout start
    med = statistics.median
    print(f"{label} updates={len(span)} span={med(span):.0f}us busy={med(busy):.0f} rollout={med(roll):.0f} "
          f"minibatches={med(mbs):.0f} lastmb->rollout={med(pre):.0f}")


if __name__ == "__main__":
    main()
