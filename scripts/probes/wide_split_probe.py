"""Where the wide update's parameters leave the oracle's with the split-bf16 GEMMs: the
Connect Four MLP update of test_gpu_wide.py::test_update_then_second_rollout (N = 64,
T = 16) with the default kernel choice (split after the first minibatch), with the exact
chains for every minibatch, and with split for every minibatch; per tensor the count of
entries outside the parameter bar, the largest |diff| and the oracle's value there.
Diagnosis only (run on the GPU box)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "burn-ppo_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np  # noqa: E402

import bppo  # noqa: E402
from bppo.host import layer_shapes  # noqa: E402
from parity_util import PARAM_ATOL, PARAM_RTOL  # noqa: E402
from test_gpu_wide import _pair  # noqa: E402


def run(mode, N=64, T=16):
    cfg, tr, ot = _pair("connect_four", N, T)
    tr.ctx.set_minibatch_kernel(mode)
    bppo.collect_rollouts(tr.ctx); ot.collect()
    bppo.compute_gae(tr.ctx); ot.gae()
    lr = bppo.schedule_get(cfg["learning_rate"], 0)
    ent = bppo.schedule_get(cfg["entropy_coef"], 0)
    bppo.ppo_update(tr.ctx, lr, ent); ot.update()
    pg, po = tr.model.get_params(), ot.params()
    rows, log = tr.ctx.minibatch_rows(), ot.minibatch_log()
    out = []
    off = 0
    for li, (i, o) in enumerate(layer_shapes(cfg)[0]):
        for kind, n in (("W", i * o), ("b", o)):
            a, b = pg[off:off + n], po[off:off + n]
            bad = np.abs(a - b) > PARAM_ATOL + PARAM_RTOL * np.abs(b)
            k = int(np.argmax(np.abs(a - b)))
            out.append({"layer": li, "kind": kind, "n": n, "bad": int(bad.sum()), "max_diff": float(np.abs(a - b).max()),
                        "at_oracle": float(b[k]), "at_dev": float(a[k])})
            off += n
    kl = [(float(r[3] / r[10]), float(o["approx_kl"])) for r, o in zip(rows, log)]
    tr.close(); ot.close()
    return {"mode": mode, "lr": lr, "tensors": out, "approx_kl": kl}


if __name__ == "__main__":
    res = [run(m) for m in (0, 1, 2)]
    for r in res:
        print(json.dumps({"mode": r["mode"], "lr": r["lr"], "bad": [(t["layer"], t["kind"], t["bad"], t["max_diff"],
                                                                      t["at_oracle"], t["at_dev"])
                                                                     for t in r["tensors"] if t["bad"]]}), flush=True)
    os.makedirs("gpurun_out", exist_ok=True)
    with open("gpurun_out/wide_split_probe.json", "w") as f:
        json.dump(res, f, indent=1)
