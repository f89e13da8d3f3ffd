"""Shared parity helpers: device (libbppo.so) vs oracle trainers on identical
seeds and the stated tolerances.

Tolerances (north_star: "fp32 returns/advantages/loss within 1e-5 relative"):
  * every UpdateMetrics field (ppo.rs:1342-1369) within 1e-5 relative to
    max(|oracle|, floor): the floor is the magnitude of the summands for the
    signed means that cancel to ~0 — policy_loss / total_loss are means of
    -A_n * ratio, floor mean|A_n| of the update's normalized advantages
    (summand_magnitude, ~0.8; its bound 1.0 where a test passes no advantages);
    approx_kl additionally to its f32 resolution 2^-24 / sqrt(B) (a mean of
    (ratio - 1) - log(ratio) per row, evaluated from ratios near 1); adv_mean_raw is a mean of raw
    advantages (floor adv_std_raw); value_mean / returns_mean (floor
    value_error_mean + |returns_mean|).  Both sides accumulate in f64 per
    minibatch, so what is left is per-row f32 rounding of the later minibatches,
    whose parameters differ in the last bits (gradient reduction order);
  * explained_variance: the reference sums in f32 sequentially
    (ppo.rs:1268-1294); at 10^6 rows that sum drifts by ~1e-3 absolute on the
    result (measured: 0.014473 vs the exact 0.013404 at B = 1,048,576).  The
    device computes it in f64 (a deliberate deviation: the metric is logged,
    it feeds nothing back).  So the device must equal the exact f64 explained
    variance of the same buffers within 1e-6, and the oracle's f32 value must
    equal a second restatement of the reference's f32 sequential sums
    (ev_f32_sequential) bit for bit;
  * parameters after Adam: rtol 1e-4 / atol 2e-5 (Adam divides by sqrt(v): a
    gradient entry near 0 moves by ~lr either way, so the parameter check is
    looser than the loss check).
"""
import numpy as np

import bppo
import oracle_ffi as O

METRICS = ("policy_loss", "value_loss", "entropy", "entropy_scaled", "approx_kl", "clip_fraction",
           "explained_variance", "total_loss", "value_mean", "returns_mean", "adv_mean_raw", "adv_std_raw",
           "adv_min_raw", "adv_max_raw", "value_error_mean", "value_error_std", "value_error_max",
           "avg_valid_actions", "entropy_valid_pct")
RTOL = 1e-5
PARAM_RTOL, PARAM_ATOL = 1e-4, 2e-5


def summand_magnitude(advantages):
    """mean |A_n| of the normalized advantages (utils.rs:80-89 over the update's rows): the
    size of the policy-loss summands -A_n * ratio (ratio ~ 1), against which the means
    policy_loss / total_loss, which cancel to ~0, are compared"""
    a = np.asarray(advantages, np.float64)
    if a.size < 2:
        return 1.0
    sd = a.std(ddof=1)
    return float(np.abs(a - a.mean()).mean() / sd) if sd > 0 else 1.0


def _floor(k, om, pl_mag):
    if k in ("policy_loss", "total_loss"):
        return pl_mag
    if k == "adv_mean_raw":
        return abs(om["adv_std_raw"])
    if k in ("value_mean", "returns_mean"):
        return abs(om["value_error_mean"]) + abs(om["returns_mean"])
    return 0.0


def ev_f64(values, returns):
    """ppo.rs:1268-1294 in f64 (population variances)."""
    v = np.asarray(values, np.float64)
    r = np.asarray(returns, np.float64)
    if v.size < 2:
        return 0.0
    vr = r.var()
    if vr < 1e-8:
        return 0.0
    return 1.0 - (r - v).var() / vr


def _seq_sum_f32(x):
    return np.cumsum(np.ascontiguousarray(x, np.float32), dtype=np.float32)[-1] if x.size else np.float32(0)


def ev_f32_sequential(values, returns):
    """ppo.rs:1268-1294 as the reference computes it: f32 iterator sums in order."""
    v = np.ascontiguousarray(values, np.float32)
    r = np.ascontiguousarray(returns, np.float32)
    n = np.float32(v.size)
    if n < 2:
        return np.float32(0)
    mr = _seq_sum_f32(r) / n
    q = (r - mr).astype(np.float32)
    vr = _seq_sum_f32(q * q) / n
    if vr < np.float32(1e-8):
        return np.float32(0)
    res = (r - v).astype(np.float32)
    mres = _seq_sum_f32(res) / n
    q = (res - mres).astype(np.float32)
    vres = _seq_sum_f32(q * q) / n
    return np.float32(np.float32(1) - np.float32(vres / vr))


def assert_metrics_close(m, om, values=None, returns=None, skip=(), rtol=RTOL, advantages=None):
    """All 19 UpdateMetrics fields plus num_updates / epochs_run.  values /
    returns / advantages: the buffers the update trained on (learner rows only
    under an opponent pool): the explained variance is taken over the first two,
    the policy-loss summand magnitude (the floor of policy_loss / total_loss) over
    the advantages; without them the floor is its bound, E|A_n| <= 1 for
    unit-variance normalized advantages."""
    pl_mag = 1.0 if advantages is None else summand_magnitude(advantages)
    # approx_kl: each row's (ratio - 1) - log(ratio) is evaluated in f32 from a ratio near 1
    # (resolution 2^-24, half an ulp of 1.0), so a mean over the update's B rows resolves
    # approx_kl only to ~2^-24 / sqrt(B) absolute, whatever its (small) size
    kl_abs = 0.0 if advantages is None else 2.0 ** -24 / np.sqrt(max(np.asarray(advantages).size, 1))
    assert m["num_updates"] == om["num_updates"], (m["num_updates"], om["num_updates"])
    assert m["epochs_run"] == om["epochs_run"], (m["epochs_run"], om["epochs_run"])
    bad = []
    for k in METRICS:
        if k in skip:
            continue
        d, o = float(m[k]), float(om[k])
        if k == "explained_variance" and values is not None:
            ex = ev_f64(values, returns)
            ref32 = float(ev_f32_sequential(values, returns))
            if abs(d - ex) > 1e-6 or o != ref32:
                bad.append((k, d, o, ex, ref32))
            continue
        if np.isnan(o) and np.isnan(d):
            continue
        tol = rtol * max(abs(o), _floor(k, om, pl_mag))
        if k == "approx_kl":
            tol = max(tol, kl_abs)
        if not abs(d - o) <= tol:
            bad.append((k, d, o, abs(d - o) / max(abs(o), 1e-30)))
    # PopArt (ppo.rs:2061-2068): NaN = None on both sides
    for k in ("value_norm_target_mean", "value_norm_target_std", "value_norm_rescale_mag"):
        if k in skip or k not in om:
            continue
        d, o = float(m[k]), float(om[k])
        if np.isnan(o) or np.isnan(d):
            if not (np.isnan(o) and np.isnan(d)):
                bad.append((k, d, o))
            continue
        if not abs(d - o) <= rtol * max(abs(o), 1.0 if k == "value_norm_target_mean" else 0.0):
            bad.append((k, d, o))
    assert not bad, bad


def assert_params_close(pg, po):
    np.testing.assert_allclose(pg, po, rtol=PARAM_RTOL, atol=PARAM_ATOL)


def bits(a):
    return np.ascontiguousarray(a, np.float32).view(np.uint32)


def oracle_train_cfg(cfg, threads=0, rank=0, world=1):
    """the oracle's TrainCfg for a bppo config dict (CartPole, Connect Four, Liar's Dice; MLP / CTDE);
    rank / world: that rank's shard of a data-parallel job (bppo.dist.shard)"""
    kind = {"cartpole": O.ENV_CARTPOLE, "connect_four": O.ENV_CONNECT_FOUR, "liars_dice": O.ENV_LIARS_DICE}[cfg["env"]]
    nr = cfg["normalize_returns"]
    if nr is None:
        nr = cfg["env"] == "cartpole"                      # main.rs:243: single-player only
    return O.train_cfg(env_kind=kind, num_envs=cfg["num_envs"], num_steps=cfg["num_steps"], seed=cfg["seed"],
                       hidden=cfg["hidden_size"], num_hidden=cfg["num_hidden"], ctde=cfg["network_type"] == "ctde",
                       relu=cfg["activation"] == "relu", critic_hidden=cfg["critic_hidden_size"] or 0,
                       critic_num_hidden=cfg["critic_num_hidden"] or 0, normalize_obs=bool(cfg["normalize_obs"]),
                       normalize_returns=bool(nr), gamma=cfg["gamma"], gae_lambda=cfg["gae_lambda"],
                       lr=bppo.schedule_get(cfg["learning_rate"], 0), ent_coef=bppo.schedule_get(cfg["entropy_coef"], 0),
                       reward_shaping=cfg["reward_shaping_coef"], num_epochs=cfg["num_epochs"],
                       num_minibatches=cfg["num_minibatches"], clip=cfg["clip_epsilon"], value_coef=cfg["value_coef"],
                       max_grad_norm=cfg["max_grad_norm"], target_kl=cfg["target_kl"], threads=threads,
                       split=bool(cfg.get("split_networks")), clip_value=bool(cfg.get("clip_value")),
                       env_seed_offset=rank * cfg["num_envs"] if world > 1 else 0,
                       rng_stream=rank if world > 1 else 0, shuffle_windows=bool(cfg.get("shuffle_windows")),
                       normalize_values=bool(cfg.get("normalize_values")))


def cartpole_pair(N, T, preset="cartpole", seed=42, init_seed=1, **kw):
    """Device trainer + oracle trainer of one CartPole config (same params, seeds)."""
    cfg = bppo.make_config(preset, num_envs=N, num_steps=T, seed=seed, **kw)
    params = bppo.orthogonal_init(cfg, seed=init_seed)
    tr = bppo.Trainer(cfg, params=params)
    nr = cfg["normalize_returns"]
    ocfg = O.train_cfg(num_envs=N, num_steps=T, seed=seed, lr=bppo.schedule_get(cfg["learning_rate"], 0),
                       ent_coef=bppo.schedule_get(cfg["entropy_coef"], 0),
                       hidden=cfg["hidden_size"], num_hidden=cfg["num_hidden"],
                       relu=cfg["activation"] == "relu", normalize_obs=bool(cfg["normalize_obs"]),
                       normalize_returns=True if nr is None else bool(nr), gamma=cfg["gamma"],
                       gae_lambda=cfg["gae_lambda"], num_epochs=cfg["num_epochs"],
                       num_minibatches=cfg["num_minibatches"], clip=cfg["clip_epsilon"],
                       value_coef=cfg["value_coef"], max_grad_norm=cfg["max_grad_norm"],
                       target_kl=cfg["target_kl"])
    ot = O.Trainer(ocfg, params)
    return cfg, tr, ot


def cmp_cartpole_rollout(tr, ot):
    b = tr.buffer
    assert np.array_equal(b.actions.reshape(-1), ot.buffer("actions", np.int32))
    assert np.array_equal(b.dones.reshape(-1), ot.buffer("dones"))
    assert np.array_equal(bits(b.observations.reshape(-1)), bits(ot.buffer("obs")))
    assert np.array_equal(bits(b.values.reshape(-1)), bits(ot.buffer("values")))
    assert np.array_equal(bits(b.log_probs.reshape(-1)), bits(ot.buffer("log_probs")))
    # return normalizer: f64 block scan vs the sequential Welford update ->
    # normalized f32 rewards equal up to rare last-ulp ties
    np.testing.assert_allclose(b.rewards.reshape(-1), ot.buffer("rewards"), rtol=2e-7, atol=0)
    assert tr.ctx.rng_pos() == ot.rng_pos()
