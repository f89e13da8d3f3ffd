"""Throughput of the multi-player workloads (SURVEY CfgC / CfgD) on one MI355X.

    python scripts/bench_wide.py --workload cfgC|cfgD [--steps K --warmup W]
                                 [--opponents K --opponent-frac F]

Not the driver's bench line (bench.py measures BASELINE.json's CfgB): this
prints one JSON line per workload with env-steps/s of a full update (rollout +
bootstrap/GAE + PPO update) and per-phase device times, for DESIGN.md."""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "burn-ppo_amd"))

WORKLOADS = {
    # configs/connect_four.toml at num_envs=16384, T=64 (opponent pool off), 6 epochs x 4 minibatches
    "cfgC": dict(preset="connect_four", num_envs=16384, num_steps=64),
    # configs/liars_dice_ctde.toml at num_envs=32768, T=128, 4 epochs x 8 minibatches
    "cfgD": dict(preset="liars_dice_ctde", num_envs=32768, num_steps=128),
    # CfgC with network_type = "cnn": the config.rs:996-1010 defaults (2 conv x 8 channels,
    # 3x3, FC 32), and a wide variant (64 / 64 channels, FC 128 x 2)
    "cfgC_cnn": dict(preset="connect_four", num_envs=16384, num_steps=64,
                     over=dict(network_type="cnn")),
    "cfgC_cnn64": dict(preset="connect_four", num_envs=16384, num_steps=64,
                       over=dict(network_type="cnn", conv_channels=[64, 64], cnn_fc_hidden_size=128,
                                 cnn_num_fc_layers=2)),
}


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--workload", default="cfgC", choices=sorted(WORKLOADS))
    p.add_argument("--steps", type=int, default=3)
    p.add_argument("--warmup", type=int, default=1)
    p.add_argument("--num-envs", type=int, default=None)
    p.add_argument("--no-kl-stop", action="store_true", help="run every epoch (target_kl off)")
    p.add_argument("--opponents", type=int, default=0,
                   help="opponent-pool rollouts (ppo.rs:537-1063) against K loaded models")
    p.add_argument("--minibatch-kernel", type=int, default=None,
                   help="bppo_set_minibatch_kernel mode: 0 default (below 32768-row minibatches exact chains + "
                        "f64 weight gradients; from 32768 rows MLP nets split-bf16 GEMMs after the first "
                        "minibatch's exact forward, CNN nets f32 split-K weight gradients), 1 exact chains + "
                        "row-ordered f64 weight gradients, 2 split-bf16 for every MLP minibatch (CNN: f32 split-K)")
    p.add_argument("--opponent-frac", type=float, default=0.25,
                   help="opponent_pool_fraction (configs/liars_dice*.toml: 0.25)")
    a = p.parse_args()
    import torch
    import bppo
    w = dict(WORKLOADS[a.workload])
    if a.num_envs:
        w["num_envs"] = a.num_envs
    over = dict(w.get("over", {}))
    if a.no_kl_stop:
        over["target_kl"] = None
    cfg = bppo.make_config(w["preset"], num_envs=w["num_envs"], num_steps=w["num_steps"], **over)
    torch.cuda.set_device(0)
    tr = bppo.Trainer(cfg, init_seed=0)
    if a.minibatch_kernel is not None:
        tr.ctx.set_minibatch_kernel(a.minibatch_kernel)
    if a.opponents:
        import numpy as np
        P = tr.ctx.num_players
        n_opp = max(1, int(w["num_envs"] * a.opponent_frac))          # main.rs:621-637
        rng = np.random.default_rng(0)
        opp = np.stack([bppo.orthogonal_init(cfg, seed=50 + k) for k in range(a.opponents)])
        lp = rng.integers(0, P, n_opp).astype(np.int32)
        po = np.where(np.arange(P)[None, :] == lp[:, None], -1,
                      rng.integers(0, a.opponents, (n_opp, P))).astype(np.int32)
        tr.ctx.set_opponents(opp, None, n_opp, lp, po, rng.integers(0, a.opponents, P - 1))
    for _ in range(a.warmup):
        tr.train_update()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ph = {"rollout": 0.0, "gae": 0.0, "update": 0.0}
    ups = 0
    for _ in range(a.steps):
        m = tr.train_update()
        ups += m["num_updates"]
        for k in ph:
            ph[k] += tr.ctx.kernel_ms(k)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    B = w["num_envs"] * w["num_steps"]
    out = {"workload": a.workload + (f"+opponents{a.opponents}@{a.opponent_frac}" if a.opponents else ""),
           "env_steps_per_sec": round(B * a.steps / dt, 1),
           "ms_per_update": round(dt / a.steps * 1000, 2), "num_envs": w["num_envs"],
           "num_steps": w["num_steps"], "minibatches_per_update": ups / a.steps,
           "phase_ms_per_update": {k: round(v / a.steps, 2) for k, v in ph.items()},
           # the reference's own names (main.rs:1092-1132) over the timed interval
           "perf": {k: round(v, 6) for k, v in bppo.perf_scalars(B * a.steps, dt, ph["rollout"], ph["gae"],
                                                                 ph["update"]).items()},
           "last": {k: round(v, 5) for k, v in m.items() if isinstance(v, float)}}
    print(json.dumps(out), flush=True)
    tr.close()


if __name__ == "__main__":
    main()
