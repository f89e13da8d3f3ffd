"""Isolated Fisher-Yates passes at CfgB size (n = 2^23, J[i] uniform in [0, i]) through
the debug hook, for a kernel trace: python scripts/fy_probe.py [reps]"""
import sys

import numpy as np

sys.path.insert(0, "burn-ppo_amd")
import bppo._lib as L  # noqa: E402

n = 1 << 23
rng = np.random.default_rng(0)
J = np.floor(rng.random(n) * (np.arange(n) + 1)).astype(np.uint32)
perm = np.zeros(n, np.uint32)
for _ in range(int(sys.argv[1]) if len(sys.argv) > 1 else 5):
    assert L.lib().bppo_debug_fisher_yates(0, J.ctypes.data, n, perm.ctypes.data) == 0
print("ok", perm[:4])
