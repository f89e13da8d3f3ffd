"""Where the 64-channel CNN update leaves the oracle's bits: one update of E epochs (E = 1..4,
connect_four.toml minibatches, N = 1024, T = 8) from identical parameters, then the
parameters and the Adam moments compared entry by entry (count of differing entries,
largest difference in ulps, per tensor).  Diagnosis only (run on the GPU box)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "burn-ppo_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np  # noqa: E402

import bppo  # noqa: E402
import oracle_ffi as O  # noqa: E402

NET = dict(num_conv_layers=2, conv_channels=[64, 64], kernel_size=3, cnn_fc_hidden_size=128, cnn_num_fc_layers=2)


def ulps(a, b):
    return np.abs(a.view(np.int32).astype(np.int64) - b.view(np.int32).astype(np.int64))


def run(epochs, mbs, N=1024, T=8, mode=None):
    cfg = bppo.make_config("connect_four", num_envs=N, num_steps=T, network_type="cnn", num_epochs=epochs,
                           num_minibatches=mbs, **NET)
    params = bppo.orthogonal_init(cfg, seed=7)
    tr = bppo.Trainer(cfg, params=params)
    if mode is not None:
        tr.ctx.set_minibatch_kernel(mode)
    ocfg = O.train_cfg(env_kind=O.ENV_CONNECT_FOUR, num_envs=N, num_steps=T, seed=cfg["seed"], hidden=128,
                       num_hidden=2, relu=True, normalize_obs=False, normalize_returns=False, gamma=cfg["gamma"],
                       gae_lambda=cfg["gae_lambda"], lr=bppo.schedule_get(cfg["learning_rate"], 0),
                       ent_coef=bppo.schedule_get(cfg["entropy_coef"], 0), num_epochs=epochs, num_minibatches=mbs,
                       clip=cfg["clip_epsilon"], value_coef=cfg["value_coef"], target_kl=cfg["target_kl"],
                       cnn=([64, 64], 3))
    ot = O.Trainer(ocfg, params)
    bppo.collect_rollouts(tr.ctx); ot.collect()
    bppo.compute_gae(tr.ctx); ot.gae()
    same_adv = bool(np.array_equal(tr.buffer.advantages.reshape(-1).view(np.uint32), ot.buffer("advantages").view(np.uint32)))
    bppo.ppo_update(tr.ctx, bppo.schedule_get(cfg["learning_rate"], 0), bppo.schedule_get(cfg["entropy_coef"], 0))
    ot.update()
    rows, log = tr.ctx.minibatch_rows(), ot.minibatch_log()
    stats = []
    for r, o in zip(rows, log):
        n = r[10]
        dev = {"policy_loss": r[0] / n, "value_loss": 0.5 * r[1] / n, "entropy": r[2] / n, "approx_kl": r[3] / n,
               "clip_fraction": r[4] / n}
        stats.append({k: float(dev[k] - o[k]) for k in dev})
    pg, po = tr.model.get_params(), ot.params()
    shapes, _ = bppo.host.layer_shapes(cfg)
    per = []
    off = 0
    for i, o in shapes:
        for n in (i * o, o):
            u = ulps(pg[off:off + n], po[off:off + n])
            per.append({"off": off, "n": n, "diff": int(np.count_nonzero(u)), "max_ulp": int(u.max())})
            off += n
    # the minibatch statistics' advantage columns (mean, std of each minibatch's advantages)
    adv_stats = [[float(x) for x in r[-4:]] for r in rows]
    tr.close(); ot.close()
    return {"epochs": epochs, "minibatches": mbs, "mode": mode, "same_adv": same_adv,
            "params_diff": int(np.count_nonzero(ulps(pg, po))), "per_tensor": per, "mb_stat_diffs": stats,
            "adv_stats": adv_stats}


if __name__ == "__main__":
    out = []
    for mode in (None, 1):
        for e in (1, 2, 3, 6):
            out.append(run(e, 4, mode=mode))
            r = out[-1]
            print(json.dumps({k: r[k] for k in ("mode", "epochs", "same_adv", "params_diff")}),
                  [(t["off"], t["diff"], t["max_ulp"]) for t in r["per_tensor"] if t["diff"]],
                  "max|mb stat diff|", max(max(abs(v) for v in d.values()) for d in r["mb_stat_diffs"]), flush=True)
    os.makedirs("gpurun_out", exist_ok=True)
    with open("gpurun_out/cnn_exact_probe.json", "w") as f:
        json.dump(out, f, indent=1)
