"""Parity of the multi-player path (Connect Four, Liar's Dice MLP and CTDE)
through libbppo.so against the CPU oracle on identical seeds.

Bit-exact: env transitions (observations, privileged obs, action masks, acting
players, rewards, dones, episode records), masked Gumbel-max actions, log-probs,
values (the MFMA GEMM forward reproduces matrixmultiply's fma chains), the main
RNG position, multiplayer GAE.  The update (gradients reduced in a different
order): every UpdateMetrics field within 1e-5 relative, parameters after Adam
within rtol 1e-4 / atol 2e-5 (tests/parity_util.py)."""
import ctypes as C

import numpy as np
import pytest

import bppo
import bppo._lib as L
import oracle_ffi as O
from parity_util import assert_metrics_close, assert_params_close
from bppo.host import shaping_schedule

pytestmark = pytest.mark.gpu

ENV = {"connect_four": (O.ENV_CONNECT_FOUR, 86, 7, 2, 0), "liars_dice": (O.ENV_LIARS_DICE, 270, 49, 4, 120)}


# --------------------------------------------------------------- VecEnv ---
@pytest.mark.parametrize("env", ["connect_four", "liars_dice"])
def test_vecenv_matches_oracle(env):
    kind, D, A, P, G = ENV[env]
    N = 300
    preset = "connect_four" if env == "connect_four" else "liars_dice_ctde"
    cfg = bppo.make_config(preset, num_envs=N, num_steps=4, reward_shaping_coef=0.05 if G else 0.0)
    ctx = bppo.Context(cfg)
    ve = bppo.VecEnv.new(ctx)
    ov = O.lib().or_vecenv_new(kind, N, cfg["seed"])
    O.lib().or_vecenv_set_shaping(ov, cfg["reward_shaping_coef"])
    obs_o = np.zeros(N * D, np.float32)
    m_o = np.zeros(N * A, np.uint8)
    pl_o = np.zeros(N, np.int32)
    g_o = np.zeros(max(N * G, 1), np.float32)
    rw = np.zeros(N * P, np.float32); dn = np.zeros(N, np.uint8)
    eps = (O.Episode * N)()
    rng = np.random.default_rng(1)
    n_done = 0
    for t in range(400):
        O.lib().or_vecenv_get_obs(ov, obs_o)
        O.lib().or_vecenv_get_masks(ov, m_o)
        O.lib().or_vecenv_get_players(ov, pl_o)
        assert np.array_equal(ve.get_observations(), obs_o), t
        assert np.array_equal(ve.get_action_masks(), m_o.astype(bool)), t
        assert np.array_equal(ve.get_current_players(), pl_o), t
        if G:
            O.lib().or_vecenv_get_priv(ov, g_o)
            assert np.array_equal(ve.get_privileged_obs(), g_o), t
        # a random VALID action per env (an invalid one now and then: the env's own rule)
        m = m_o.reshape(N, A).astype(bool)
        a = np.array([rng.choice(np.flatnonzero(row)) for row in m], np.int32)
        bad = rng.random(N) < 0.002
        a[bad] = rng.integers(0, A, bad.sum())
        o, r, d, ep = ve.step(a)
        ne = O.lib().or_vecenv_step(ov, a, obs_o, rw, dn, eps, N)
        assert np.array_equal(o, obs_o), t
        assert np.array_equal(r.reshape(-1), rw), t
        assert np.array_equal(d, dn.astype(bool)), t
        assert len(ep) == ne
        for i, e in enumerate(ep):
            assert e["env_index"] == eps[i].env_index and e["length"] == eps[i].length
            assert np.array_equal(np.float32(e["total_rewards"]), np.float32(eps[i].total_rewards[:P]))
        n_done += int(d.sum())
    assert n_done > 50
    O.lib().or_vecenv_free(ov)
    ctx.close()


# -------------------------------------------------------------- rollout ---
def _pair(env, N, T, seed=42, ctde=None, **kw):
    kind, D, A, P, G = ENV[env]
    if env == "connect_four":
        cfg = bppo.make_config("connect_four", num_envs=N, num_steps=T, seed=seed, **kw)
    else:
        cfg = bppo.make_config("liars_dice_ctde", num_envs=N, num_steps=T, seed=seed, **kw)
        if ctde is False:
            cfg.update(network_type="mlp", hidden_size=128)
    params = bppo.orthogonal_init(cfg, seed=5)
    tr = bppo.Trainer(cfg, params=params)
    is_ctde = cfg["network_type"] == "ctde"
    ocfg = O.train_cfg(env_kind=kind, num_envs=N, num_steps=T, seed=seed, hidden=cfg["hidden_size"],
                       num_hidden=cfg["num_hidden"], ctde=is_ctde, relu=cfg["activation"] == "relu",
                       critic_hidden=cfg["critic_hidden_size"] or 0,
                       critic_num_hidden=cfg["critic_num_hidden"] or 0,
                       normalize_obs=bool(cfg["normalize_obs"]),
                       normalize_returns=bool(cfg["normalize_returns"]), gamma=cfg["gamma"], gae_lambda=cfg["gae_lambda"],
                       lr=bppo.schedule_get(cfg["learning_rate"], 0),
                       ent_coef=bppo.schedule_get(cfg["entropy_coef"], 0),
                       reward_shaping=bppo.schedule_get(shaping_schedule(cfg), 0), num_epochs=cfg["num_epochs"],
                       num_minibatches=cfg["num_minibatches"], clip=cfg["clip_epsilon"],
                       value_coef=cfg["value_coef"], target_kl=cfg["target_kl"])
    ot = O.Trainer(ocfg, params)
    return cfg, tr, ot


def _bits(a):
    return np.ascontiguousarray(a, np.float32).view(np.uint32)


def _cmp_rollout(env, tr, ot, rew_rtol=0.0):
    kind, D, A, P, G = ENV[env]
    b = tr.buffer
    assert np.array_equal(b.acting_players.reshape(-1), ot.buffer("players", np.int32))
    assert np.array_equal(_bits(b.observations.reshape(-1)), _bits(ot.buffer("obs")))
    assert np.array_equal(b.action_masks.reshape(-1), ot.buffer("masks"))
    if G and tr.model.is_ctde():
        assert np.array_equal(_bits(b.privileged_obs.reshape(-1)), _bits(ot.buffer("priv")))
    assert np.array_equal(b.actions.reshape(-1), ot.buffer("actions", np.int32))
    assert np.array_equal(_bits(b.values.reshape(-1)), _bits(ot.buffer("values")))
    assert np.array_equal(_bits(b.log_probs.reshape(-1)), _bits(ot.buffer("log_probs")))
    assert np.array_equal(b.dones.reshape(-1), ot.buffer("dones"))
    if rew_rtol:
        # return normalizer: f64 Welford block scan vs the sequential update
        # (merge order) -> normalized rewards identical up to rare last-ulp ties
        np.testing.assert_allclose(b.rewards.reshape(-1), ot.buffer("rewards"), rtol=rew_rtol, atol=0)
        np.testing.assert_allclose(b.all_rewards.reshape(-1), ot.buffer("all_rewards"), rtol=rew_rtol, atol=0)
    else:
        assert np.array_equal(_bits(b.rewards.reshape(-1)), _bits(ot.buffer("rewards")))
        assert np.array_equal(_bits(b.all_rewards.reshape(-1)), _bits(ot.buffer("all_rewards")))
    assert tr.ctx.rng_pos() == ot.rng_pos()


@pytest.mark.parametrize("ctde", [None, False])
def test_liars_dice_shaping_schedule(ctde):
    """reward_shaping_coef as a Schedule (liars_dice.rs:164, 535; main.rs:720-727):
    each rollout uses coef.get(global_step) set through VecEnv::set_step; the
    oracle gets the same value from its own Schedule::get restatement."""
    N, T = 48, 16
    sched = [(0.2, 0), (0.05, 2 * N * T), (0.0, 4 * N * T)]
    cfg, tr, ot = _pair("liars_dice", N, T, ctde=ctde, reward_shaping_coef=sched)
    v = np.array([a for a, _ in sched]); st = np.array([b for _, b in sched], np.uint64)
    coefs = []
    for k in range(4):
        step = k * N * T + (N * T // 2 if k == 3 else 0)
        tr.vec_env.set_step(step)
        c = O.lib().or_schedule_get(v.ctypes.data, st.ctypes.data, len(v), step)
        assert c == bppo.schedule_get(sched, step)
        coefs.append(c)
        O.lib().or_trainer_set_shaping(ot.h, c)
        bppo.collect_rollouts(tr.ctx); ot.collect()
        _cmp_rollout("liars_dice", tr, ot)
    assert len(set(coefs)) == 4
    tr.close(); ot.close()


def test_shaping_schedule_rejects_negative_initial():
    cfg = bppo.make_config("liars_dice_ctde", num_envs=8, num_steps=4)
    tr = bppo.Trainer(cfg)
    with pytest.raises(bppo.BppoError):
        tr.ctx.set_reward_shaping_schedule([(-0.1, 0), (0.1, 100)])
    tr.ctx.set_reward_shaping_schedule([(0.0, 0), (-0.1, 100)])    # only the initial value is validated
    tr.close()
    with pytest.raises(bppo.BppoError):
        bppo.Trainer(bppo.make_config("liars_dice_ctde", num_envs=8, num_steps=4, reward_shaping_coef=-1.0))


CASES = [("connect_four", 64, 16, None), ("liars_dice", 48, 16, None), ("liars_dice", 40, 12, False)]


@pytest.mark.parametrize("env,N,T,ctde", CASES)
def test_rollout_and_gae_bit_exact(env, N, T, ctde):
    cfg, tr, ot = _pair(env, N, T, ctde=ctde)
    info = bppo.collect_rollouts(tr.ctx)
    n_eps = ot.collect()
    _cmp_rollout(env, tr, ot)
    assert info.episodes == n_eps
    bppo.compute_gae(tr.ctx)
    ot.gae()
    assert np.array_equal(_bits(tr.ctx.buffer("last_v_pp")), _bits(ot.buffer("last_v_pp")))
    assert np.array_equal(_bits(tr.buffer.advantages.reshape(-1)), _bits(ot.buffer("advantages")))
    assert np.array_equal(_bits(tr.buffer.returns.reshape(-1)), _bits(ot.buffer("returns")))
    tr.close(); ot.close()


@pytest.mark.parametrize("env,N,T,ctde", CASES)
def test_update_then_second_rollout(env, N, T, ctde):
    cfg, tr, ot = _pair(env, N, T, ctde=ctde)
    bppo.collect_rollouts(tr.ctx); ot.collect()
    bppo.compute_gae(tr.ctx); ot.gae()
    lr = bppo.schedule_get(cfg["learning_rate"], 0)
    ent = bppo.schedule_get(cfg["entropy_coef"], 0)
    m = bppo.ppo_update(tr.ctx, lr, ent)
    om = ot.update()
    assert tr.ctx.rng_pos() == ot.rng_pos()
    assert_metrics_close(m, om, values=ot.buffer("values"), returns=ot.buffer("returns"), advantages=ot.buffer("advantages"))
    assert_params_close(tr.model.get_params(), ot.params())
    # the next rollout from the oracle's parameters is bit-identical again
    tr.model.set_params(ot.params())
    bppo.collect_rollouts(tr.ctx); ot.collect()
    _cmp_rollout(env, tr, ot)
    tr.close(); ot.close()


def test_forward_matches_oracle_ctde():
    cfg = bppo.make_config("liars_dice_ctde", num_envs=16, num_steps=2)
    params = bppo.orthogonal_init(cfg, seed=9)
    tr = bppo.Trainer(cfg, params=params)
    rng = np.random.default_rng(0)
    obs = (rng.random((300, 270)) < 0.1).astype(np.float32)
    priv = rng.random((300, 120)).astype(np.float32)
    lg, v = tr.model.forward(obs, priv)
    d = O.ctde_desc(270, 120, 49, 256, 2, 512, 3)
    lo, vo = O.net_forward(d, params, obs, priv)
    assert np.array_equal(_bits(lg), _bits(lo))
    assert np.array_equal(_bits(v.reshape(-1)), _bits(vo))
    tr.close()


# tanh hidden layers (config.rs:990-992 default) on the GEMM path: the rollout
# stays bit-exact, the update within the same tolerance as relu
TANH_CASES = [("connect_four", 64, 12, None), ("liars_dice", 40, 10, None)]


@pytest.mark.parametrize("env,N,T,ctde", TANH_CASES)
def test_tanh_rollout_update_second_rollout(env, N, T, ctde):
    cfg, tr, ot = _pair(env, N, T, ctde=ctde, activation="tanh")
    bppo.collect_rollouts(tr.ctx); ot.collect()
    _cmp_rollout(env, tr, ot)
    bppo.compute_gae(tr.ctx); ot.gae()
    assert np.array_equal(_bits(tr.buffer.advantages.reshape(-1)), _bits(ot.buffer("advantages")))
    m = bppo.ppo_update(tr.ctx, bppo.schedule_get(cfg["learning_rate"], 0), bppo.schedule_get(cfg["entropy_coef"], 0))
    om = ot.update()
    assert_metrics_close(m, om, values=ot.buffer("values"), returns=ot.buffer("returns"), advantages=ot.buffer("advantages"))
    assert_params_close(tr.model.get_params(), ot.params())
    tr.model.set_params(ot.params())
    bppo.collect_rollouts(tr.ctx); ot.collect()
    _cmp_rollout(env, tr, ot)
    tr.close(); ot.close()


# observation + return normalizers on the multi-player path (main.rs:235-254:
# off by default for P > 1, available by config): lagged obs stats, per
# (env, player) rolling returns for the acting player, the normalized acting
# reward in all_rewards
NORM_CASES = [("connect_four", 64, 12, None), ("liars_dice", 48, 10, None), ("liars_dice", 40, 8, False)]


@pytest.mark.parametrize("env,N,T,ctde", NORM_CASES)
def test_normalizers_rollout_update_second_rollout(env, N, T, ctde):
    kind, D, A, P, G = ENV[env]
    cfg, tr, ot = _pair(env, N, T, ctde=ctde, normalize_obs=True, normalize_returns=True)
    # first rollout: obs stats still empty (count < 2), rewards normalized from step 1
    bppo.collect_rollouts(tr.ctx); ot.collect()
    _cmp_rollout(env, tr, ot, rew_rtol=2e-7)
    m, v, c = tr.ctx.obs_norm()
    mo, vo, co = ot.obs_norm_state(D)
    assert c == co == N * T
    np.testing.assert_allclose(m, mo, rtol=1e-12, atol=1e-15)
    np.testing.assert_allclose(v, vo, rtol=1e-10, atol=1e-12)
    mvc, rets = tr.ctx.ret_norm()
    omvc, orets = ot.ret_norm_state(returns=True)
    assert np.array_equal(rets, orets)
    np.testing.assert_allclose(mvc, omvc, rtol=1e-12)
    bppo.compute_gae(tr.ctx); ot.gae()
    np.testing.assert_allclose(tr.buffer.advantages.reshape(-1), ot.buffer("advantages"), rtol=1e-5, atol=1e-6)
    m_ = bppo.ppo_update(tr.ctx, bppo.schedule_get(cfg["learning_rate"], 0), bppo.schedule_get(cfg["entropy_coef"], 0))
    om = ot.update()
    assert_metrics_close(m_, om, values=ot.buffer("values"), returns=ot.buffer("returns"), advantages=ot.buffer("advantages"))
    # second rollout from the oracle's params and normalizer state: normalized
    # observations (now count >= 2) and rewards bit-exact again
    tr.model.set_params(ot.params())
    mo, vo, co = ot.obs_norm_state(D)
    tr.ctx.set_obs_norm(mo, vo, co)
    tr.ctx.set_ret_norm(omvc, orets)
    bppo.collect_rollouts(tr.ctx); ot.collect()
    _cmp_rollout(env, tr, ot, rew_rtol=2e-7)
    tr.close(); ot.close()


# ------------------------------------------------------- opponent pool ---
# collect_rollouts_with_opponents (ppo.rs:537-1063) + the learner-row filter of
# ppo_update (ppo.rs:1696-1753).  Oracle and device get the same opponent
# models (one with its own obs normalizer), seats and current opponents.
def _opponent_setup(cfg, tr, ot, env, n_opp, K, seed=3):
    kind, D, A, P, G = ENV[env]
    rng = np.random.default_rng(seed)
    params = np.stack([bppo.orthogonal_init(cfg, seed=100 + k) for k in range(K)])
    norms = [None] * K
    norms[K - 1] = (rng.normal(size=D) * 0.1, (rng.random(D) + 0.5) * 500.0, 500.0)
    lp = rng.integers(0, P, n_opp).astype(np.int32)
    po = np.full((n_opp, P), -1, np.int32)
    for e in range(n_opp):
        for p in range(P):
            if p != lp[e]:
                po[e, p] = rng.integers(0, K)
    co = rng.integers(0, K, P - 1).astype(np.int32)
    tr.ctx.set_opponents(params, norms, n_opp, lp, po, co)
    ot.set_opponents(params, norms, n_opp, lp, po.reshape(-1), co)
    return P


OPP_CASES = [("connect_four", 64, 16, None, 40, 2, False), ("liars_dice", 48, 12, None, 48, 3, False),
             ("liars_dice", 40, 10, False, 25, 2, False), ("connect_four", 64, 16, None, 40, 3, True),
             ("liars_dice", 48, 10, None, 30, 2, True)]


@pytest.mark.parametrize("env,N,T,ctde,n_opp,K,norm", OPP_CASES)
def test_opponent_pool_rollout_update_bit_exact(env, N, T, ctde, n_opp, K, norm):
    kw = dict(normalize_obs=True, normalize_returns=True) if norm else {}
    cfg, tr, ot = _pair(env, N, T, ctde=ctde, **kw)
    P = _opponent_setup(cfg, tr, ot, env, n_opp, K)
    for rnd in range(2):
        if norm and rnd:                       # layered: the oracle's normalizer state
            kind, D, A, P_, G = ENV[env]
            tr.ctx.set_obs_norm(*ot.obs_norm_state(D))
            tr.ctx.set_ret_norm(*ot.ret_norm_state(returns=True))
        bppo.collect_rollouts(tr.ctx); ot.collect()
        _cmp_rollout(env, tr, ot, rew_rtol=2e-7 if norm else 0.0)   # includes the main RNG position
        assert np.array_equal(tr.ctx.buffer("valid"), ot.buffer("valid"))
        lp, po = tr.ctx.opponent_envs()
        olp, opo = ot.opponent_envs(n_opp, P)
        assert np.array_equal(lp, olp) and np.array_equal(po.reshape(-1), opo)
        v = tr.ctx.buffer("valid").reshape(T, N)
        assert (n_opp == N or v[:, n_opp:].min() == 1.0) and 0.0 < v[:, :n_opp].mean() < 1.0
        bppo.compute_gae(tr.ctx); ot.gae()
        if norm:
            np.testing.assert_allclose(tr.buffer.advantages.reshape(-1), ot.buffer("advantages"), rtol=1e-5, atol=1e-6)
        else:
            assert np.array_equal(_bits(tr.buffer.advantages.reshape(-1)), _bits(ot.buffer("advantages")))
        lr = bppo.schedule_get(cfg["learning_rate"], 0)
        ent = bppo.schedule_get(cfg["entropy_coef"], 0)
        m = bppo.ppo_update(tr.ctx, lr, ent)
        om = ot.update()
        assert tr.ctx.rng_pos() == ot.rng_pos()     # shuffles over the learner rows only
        vm = ot.buffer("valid") > 0.5
        assert_metrics_close(m, om, values=ot.buffer("values")[vm], returns=ot.buffer("returns")[vm], advantages=ot.buffer("advantages")[vm])
        assert_params_close(tr.model.get_params(), ot.params())
        tr.model.set_params(ot.params())
    tr.close(); ot.close()
