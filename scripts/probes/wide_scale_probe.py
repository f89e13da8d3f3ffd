"""tests/test_gpu_scale.py::test_wide_at_full_gemm_tiles[liars_dice-1024-8-False] under kernel
variants: the update's metrics and parameters against the oracle minibatch by minibatch
(approx_kl, value_loss, the largest parameter difference).  Diagnosis only (GPU box)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "burn-ppo_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np  # noqa: E402

import bppo  # noqa: E402
from test_gpu_scale import _update_pair, wide_pair  # noqa: E402


def run(mode):
    cfg, tr, ot = wide_pair("liars_dice", 1024, 8, ctde=False)
    if mode is not None:
        tr.ctx.set_minibatch_kernel(mode)
    bppo.collect_rollouts(tr.ctx); ot.collect()
    bppo.compute_gae(tr.ctx); ot.gae()
    m, om, _ = _update_pair(cfg, tr, ot, inject=False)
    rows, log = tr.ctx.minibatch_rows(), ot.minibatch_log()
    kl = [(float(r[3] / r[10]), float(o["approx_kl"])) for r, o in zip(rows, log)]
    first_bad = next((k for k, (a, b) in enumerate(kl) if abs(a - b) > 1e-5 * abs(b)), None)
    pd = float(np.abs(tr.model.get_params() - ot.params()).max())
    tr.close(); ot.close()
    return {"mode": mode, "approx_kl": (float(m["approx_kl"]), float(om["approx_kl"])), "first_mb_kl_off": first_bad,
            "kl_rows": kl, "param_max_diff": pd}


if __name__ == "__main__":
    out = [run(m) for m in (None, 1)]
    for r in out:
        print(json.dumps({k: r[k] for k in ("mode", "approx_kl", "first_mb_kl_off", "param_max_diff")}), flush=True)
    os.makedirs("gpurun_out", exist_ok=True)
    with open("gpurun_out/wide_scale_probe.json", "w") as f:
        json.dump(out, f, indent=1)
