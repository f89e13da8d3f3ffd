"""Single-minibatch gradient of the 64-channel CNN against the oracle's from identical parameters,
entry by entry, per tensor, for the default weight-gradient sums (f64 MFMA) and the row-ordered
ones (bppo_set_minibatch_kernel 1); and the parameters after 1 and 2 Adam steps.  Diagnosis."""
import ctypes as C
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "burn-ppo_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np  # noqa: E402

import bppo  # noqa: E402
import oracle_ffi as O  # noqa: E402
from cnn_exact_probe import NET, ulps  # noqa: E402


def pair(N, T, epochs, mbs, mode):
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
    return cfg, params, tr, O.Trainer(ocfg, params)


def per_tensor(cfg, a, b):
    shapes, _ = bppo.host.layer_shapes(cfg)
    out, off = [], 0
    for i, o in shapes:
        for n in (i * o, o):
            u = ulps(a[off:off + n], b[off:off + n])
            if u.any():
                out.append((off, n, int(np.count_nonzero(u)), int(u.max())))
            off += n
    return out


def grad_case(mode, N=1024, T=8):
    cfg, p0, tr, ot = pair(N, T, 1, 1, mode)
    bppo.collect_rollouts(tr.ctx); ot.collect()
    bppo.compute_gae(tr.ctx); ot.gae()
    bppo.ppo_update(tr.ctx, bppo.schedule_get(cfg["learning_rate"], 0), bppo.schedule_get(cfg["entropy_coef"], 0))
    g = tr.ctx.buffer("grad")
    B = N * T
    d = O.cnn_desc(7, [64, 64], 3, 128, 2)
    adv = ot.buffer("advantages")
    advn = np.zeros(B, np.float32)
    st = [C.c_float() for _ in range(4)]
    O.lib().or_normalize_advantages(adv, B, advn, *[C.byref(x) for x in st])
    go = np.zeros(d.n_params, np.float32)
    ms = O.MbStats()
    pc = O.ppo_cfg(num_epochs=1, num_minibatches=1, clip=cfg["clip_epsilon"], value_coef=cfg["value_coef"])
    masks = ot.buffer("masks")
    O.lib().or_minibatch_loss_grad(C.byref(d), p0, B, ot.buffer("obs"), None, ot.buffer("actions", np.int32),
                                   ot.buffer("log_probs"), advn, ot.buffer("returns"), ot.buffer("values"),
                                   masks.ctypes.data, C.byref(pc), bppo.schedule_get(cfg["entropy_coef"], 0), go,
                                   C.byref(ms))
    ot.update()
    res = {"mode": mode, "grad_diff": per_tensor(cfg, g, go),
           "params_after_1_step": per_tensor(cfg, tr.model.get_params(), ot.params())}
    tr.close(); ot.close()
    return res


def steps_case(mode, mbs, N=1024, T=8):
    cfg, p0, tr, ot = pair(N, T, 1, mbs, mode)
    bppo.collect_rollouts(tr.ctx); ot.collect()
    bppo.compute_gae(tr.ctx); ot.gae()
    bppo.ppo_update(tr.ctx, bppo.schedule_get(cfg["learning_rate"], 0), bppo.schedule_get(cfg["entropy_coef"], 0))
    ot.update()
    res = {"mode": mode, "minibatches": mbs, "params": per_tensor(cfg, tr.model.get_params(), ot.params())}
    tr.close(); ot.close()
    return res


if __name__ == "__main__":
    out = []
    for mode in (None, 1):
        out.append(grad_case(mode))
        print(json.dumps(out[-1]), flush=True)
        for mbs in (2, 4):
            out.append(steps_case(mode, mbs))
            print(json.dumps(out[-1]), flush=True)
    os.makedirs("gpurun_out", exist_ok=True)
    with open("gpurun_out/cnn_grad_probe.json", "w") as f:
        json.dump(out, f, indent=1)
