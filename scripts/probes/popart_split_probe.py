"""The Liar's Dice CTDE PopArt update (tests/test_gpu_popart.py::test_popart_multiplayer
[liars_dice-48-12-None]) minibatch by minibatch against the oracle, kernel modes 0 / 1 / 2:
where the split-bf16 GEMMs leave the oracle's statistics.  Diagnosis only (GPU box)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "burn-ppo_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np  # noqa: E402

import bppo  # noqa: E402
from test_gpu_popart import _wide  # noqa: E402

KEYS = ["policy_loss", "value_loss", "entropy", "approx_kl", "clip_fraction", "value_mean", "returns_mean"]


def run(mode, normalize_values=True):
    cfg, tr, ot = _wide("liars_dice", 48, 12, ctde=None, **({} if normalize_values else {}))
    if not normalize_values:
        pass
    tr.ctx.set_minibatch_kernel(mode)
    lr = bppo.schedule_get(cfg["learning_rate"], 0)
    ent = bppo.schedule_get(cfg["entropy_coef"], 0)
    bppo.collect_rollouts(tr.ctx); ot.collect()
    bppo.compute_gae(tr.ctx); ot.gae()
    bppo.ppo_update(tr.ctx, lr, ent); ot.update()
    rows, log = tr.ctx.minibatch_rows(), ot.minibatch_log()
    out = []
    for k, (r, o) in enumerate(zip(rows, log)):
        n = r[10]
        dev = {"policy_loss": r[0] / n, "value_loss": 0.5 * r[1] / n, "entropy": r[2] / n, "approx_kl": r[3] / n,
               "clip_fraction": r[4] / n, "value_mean": r[5] / n, "returns_mean": r[6] / n}
        out.append({"mb": k, "n": float(n), **{f: (float(dev[f]), float(o[f])) for f in KEYS}})
    pg, po = tr.model.get_params(), ot.params()
    d = np.abs(pg - po)
    tr.close(); ot.close()
    return {"mode": mode, "rows": out, "param_max_diff": float(d.max()), "param_argmax": int(d.argmax())}


if __name__ == "__main__":
    res = [run(m) for m in (1, 0, 2)]
    for r in res:
        print("mode", r["mode"], "param max diff", r["param_max_diff"], "at", r["param_argmax"])
        for row in r["rows"][:10]:
            print("  mb", row["mb"], row["n"], {f: (round(row[f][0], 6), round(row[f][1], 6)) for f in ("value_loss", "value_mean", "policy_loss")})
    os.makedirs("gpurun_out", exist_ok=True)
    with open("gpurun_out/popart_split_probe.json", "w") as f:
        json.dump(res, f, indent=1)
