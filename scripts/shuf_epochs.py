"""per-epoch walk times and meet checkpoints from a BPPO_SHUFFLE_DEBUG=1 log
   python3 scripts/shuf_epochs.py LOG..."""
import collections
import re
import sys

for path in sys.argv[1:]:
    ep, met = collections.defaultdict(list), collections.defaultdict(list)
    for line in open(path):
        m = re.search(r'epoch (\d+) end=\d+ met=(-?\d+) segs=\d+ \(([\d.]+) ms\)', line)
        if m:
            ep[int(m.group(1))].append(float(m.group(3)))
            met[int(m.group(1))].append(int(m.group(2)))
    print(path)
    for e in sorted(ep):
        print(f"  epoch {e}: mean {sum(ep[e]) / len(ep[e]):.2f} ms  {[round(x, 1) for x in ep[e]]}  met {met[e]}")
