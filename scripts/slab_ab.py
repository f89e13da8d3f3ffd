"""Parameter digest after a few CfgB-shaped updates, for A/B of build variants that
must be bit-identical (e.g. BPPO_SLAB_TWO_PASS=1 vs the fused slab reduction):
    python scripts/slab_ab.py [updates] [num_envs]"""
import hashlib
import sys

import numpy as np

sys.path.insert(0, "burn-ppo_amd")
import bppo  # noqa: E402

n_up = int(sys.argv[1]) if len(sys.argv) > 1 else 4
n_env = int(sys.argv[2]) if len(sys.argv) > 2 else 16384
cfg = bppo.make_config("cartpole", num_envs=n_env, num_steps=128)
tr = bppo.Trainer(cfg, init_seed=0)
for _ in range(n_up):
    tr.train_update()
p = np.ascontiguousarray(tr.model.get_params(), dtype=np.float32)
print("params", p.size, "sha256", hashlib.sha256(p.tobytes()).hexdigest()[:32])
